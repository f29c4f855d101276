#!/usr/bin/env python3
"""Per-tile fixed cost of the 256x256 GEMM: forward GEMM (bias+relu, bf16 out) at fixed M, N over
several K; the slope is the main loop's cost per K, the intercept the per-dispatch fixed cost
(prologue + epilogue + tail).  One JSON line per K plus a fit line."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from euromillioner_amd.ops import linear as LIN

    M, N = int(os.environ.get("KSCAN_M", 16384)), int(os.environ.get("KSCAN_N", 8192))
    g = torch.Generator(device="cuda").manual_seed(0)
    res = []
    for K in (1024, 2048, 4096, 8192, 16384):
        x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
        b = torch.zeros(N, device="cuda")
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        fn = lambda: LIN.linear_fwd(x, w, b, "relu", out=y)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = max(5, int(4e10 / (2.0 * M * N * K)))
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        res.append((K, ms))
        print(json.dumps({"M": M, "N": N, "K": K, "ms": round(ms, 4), "tflops": round(2.0 * M * N * K / ms / 1e9, 1)}),
              flush=True)
    (k0, t0), (k1, t1) = res[-2], res[-1]
    slope = (t1 - t0) / (k1 - k0)
    fixed = t1 - slope * k1
    tiles = (M // 256) * (N // 256)
    print(json.dumps({"ms_per_1k_K": round(slope * 1024, 4), "fixed_ms": round(fixed, 4),
                      "fixed_us_per_tile_wave": round(fixed * 1e3 / max(1, tiles / 256), 2)}))


if __name__ == "__main__":
    main()
