#!/usr/bin/env python3
"""Fused v4 train kernel time vs batch (fixed prologue/epilogue cost = intercept of the fit).

Times FM.train_partials alone (no Adam) with CUDA events at several batch sizes on the GPU."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from euromillioner_amd.data.synthetic import generate_draws
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.ops import fused_mlp as FM

    nums, _ = generate_draws((1 << 21) + 1, seed=1, planted=0.9, native=True)
    draws = FusedSmallMLP.prepare(torch.from_numpy(nums).cuda())
    m = FusedSmallMLP("cuda", lr=1e-3)
    xs, ys = [], []
    for lb in (12, 14, 15, 16, 17, 18, 19, 20, 21):
        B = 1 << lb
        for _ in range(3):
            FM.train_partials(draws, B, m.img, m.slabs, m.loss_slabs, loss="softmax")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            FM.train_partials(draws, B, m.img, m.slabs, m.loss_slabs, loss="softmax")
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        xs.append(B)
        ys.append(us)
        print(f"B={B:8d}  {us:8.2f} us  {B / us * 1e-3:7.3f} G samples/s", flush=True)
    a, b = np.polyfit(np.array(xs[-4:], float), np.array(ys[-4:]), 1)
    print(f"fit over the largest 4: {b:.2f} us fixed + {a * 1e6:.3f} us per 1M samples")


if __name__ == "__main__":
    main()
