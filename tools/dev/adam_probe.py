#!/usr/bin/env python3
"""Where the Adam slab kernel's time goes: the same launch with fewer slabs reduced (the slab
buffer is the real one; nslab only shortens the reduction), next to a trivial one-block kernel
as the per-launch floor in a hipGraph of 10 launches.  One JSON line."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.step_parts import timed_graph  # noqa: E402


def main():
    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.ops import fused_mlp as FM

    B = 1 << 20
    draws = generate_masks(B + 16, seed=1, planted=0.9)
    m = FusedSmallMLP("cuda", lr=1e-3)
    nslab = FM.train_partials(draws, B, m.img, m.slabs, m.loss_slabs, loss="softmax")
    res = {"nslab": nslab}
    tiny = torch.zeros(64, device="cuda")
    res["floor_us"] = timed_graph(lambda: tiny.add_(1.0))
    for n in sorted({nslab, nslab // 2, nslab // 4, 16, 1}, reverse=True):
        res[f"adam_{n}_us"] = timed_graph(lambda n=n: FM.adam_slab(
            m.slabs, n, 1.0 / B, m.params, m.m, m.v, m.hp, m.state, mode=0, img=m.img,
            loss_slabs=m.loss_slabs, loss_out=m.loss_out, loss_scale=1.0 / B))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
