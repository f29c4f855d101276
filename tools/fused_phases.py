#!/usr/bin/env python3
"""Per-phase cycle breakdown of the fused v4 train kernel (diagnostic build only).

Build with `python -m euromillioner_amd._build --define V4_STAMPS=1`, then run this on the GPU: it
trains a few steps at the benchmark batch and prints, per wave role, the share of s_memtime cycles
spent in each phase of a 32-sample tile (csrc/mlp_fused.hip, V4Stamps).  Rebuild without the define
afterwards -- the stamps drain LDS counters at every mark and slow the kernel down."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["F1+relu+Himg", "F2 own", "wait H", "F2 partner+Ximg", "loss part1", "wait stats", "dz+pack+D2",
          "wait dz", "B1+mask", "dW+db2"]
if os.environ.get("EM_FUSED_V5") == "1":  # v5 round phases (csrc/mlp_fused.hip, mlp_fused_train_v5_kernel)
    PHASES = ["A (own tile)", "wait 1", "B1 dW2", "wait 2", "dump", "wait 3", "B2 dW1", "wait 4", "-", "-"]


def main():
    from euromillioner_amd.data.synthetic import generate_draws
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.ops import fused_mlp as FM

    nums, _ = generate_draws((1 << 21) + 1, seed=1, planted=0.9, native=True)
    draws = FusedSmallMLP.prepare(torch.from_numpy(nums).cuda())
    m = FusedSmallMLP("cuda", lr=1e-3)
    B = 1 << 20
    for i in range(3):
        m.step(draws, B, offset=0)
    torch.cuda.synchronize()
    m.slabs.zero_()
    nslab = FM.train_partials(draws, B, m.img, m.slabs, m.loss_slabs, loss="softmax")
    torch.cuda.synchronize()
    st = m.slabs[:nslab, FM.P_TOTAL:FM.P_TOTAL + 128].reshape(nslab, 8, 16)[:, :, :10].double().cpu().numpy()
    if not st.any():
        raise SystemExit("no stamps recorded: build with --define V4_STAMPS=1")
    raw = m.slabs[:nslab, FM.P_TOTAL + 128:FM.P_TOTAL + 132].contiguous().view(torch.int32).cpu().numpy()
    if not raw.any():
        raw = np.zeros((nslab, 4), np.int32)
    t = raw.astype(np.int64) & 0xFFFFFFFF
    t -= t[:, 0].min()
    us = t / 100.0  # s_memrealtime ticks at 100 MHz
    print(f"block wall clock (us, {nslab} blocks): entry spread {us[:, 0].max():.2f}; "
          f"prologue {np.mean(us[:, 1] - us[:, 0]):.2f}; loop {np.mean(us[:, 2] - us[:, 1]):.2f} "
          f"(max {np.max(us[:, 2] - us[:, 1]):.2f}); dW fold {np.mean(us[:, 3] - us[:, 2]):.2f}; "
          f"first entry -> last fold {us[:, 3].max():.2f}")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    FM.train_partials(draws, B, m.img, m.slabs, m.loss_slabs, loss="softmax")
    ev1.record()
    torch.cuda.synchronize()
    print(f"kernel (event) {ev0.elapsed_time(ev1) * 1e3:.2f} us")
    for role in (0, 1):
        v = st[:, role::2, :].reshape(-1, 10).mean(0)
        tot = v.sum()
        print(f"role {role}: {tot / 1e3:.1f} k cycles per wave over the launch")
        for name, x in zip(PHASES, v):
            print(f"   {name:18s} {x / tot * 100:5.1f} %   {x / 1e3:8.1f} k")


if __name__ == "__main__":
    main()
