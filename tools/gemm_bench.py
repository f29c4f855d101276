#!/usr/bin/env python3
"""K1-K3 GEMM throughput vs torch.matmul (hipBLASLt) on the wide-MLP shapes.

    python tools/gemm_bench.py [--batch 65536] [--hidden 8192] [--iters 20]

Prints one JSON line per (pass, shape): ours vs library TFLOP/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--hidden", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cases", default="", help="comma-separated case names (default: all)")
    ap.add_argument("--no-lib", action="store_true", help="skip the library (torch/hipBLASLt) timing")
    a = ap.parse_args()
    from euromillioner_amd.ops import linear as LIN

    B, H = a.batch, a.hidden
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, H, device=dev, generator=g).bfloat16()
    w = (torch.randn(H, H, device=dev, generator=g) / H ** 0.5).bfloat16()
    bias = torch.zeros(H, device=dev)
    y = torch.empty(B, H, dtype=torch.bfloat16, device=dev)
    gw = torch.empty(H, H, dtype=torch.float32, device=dev)
    x64 = torch.randn(B, 64, device=dev, generator=g).bfloat16()
    w1 = torch.randn(H, 64, device=dev, generator=g).bfloat16()
    w3 = torch.randn(64, H, device=dev, generator=g).bfloat16()
    y64 = torch.empty(B, 64, dtype=torch.float32, device=dev)
    wt = LIN.transpose(w)
    xt = LIN.transpose(x)
    ct = torch.empty(H, B, dtype=torch.bfloat16, device=dev)
    bits = LIN.relu_bits(B, H, dev)
    colpart = torch.empty((B // 128) * H, dtype=torch.float32, device=dev)
    cases = [
        ("fwd_hidden_ct", 2.0 * B * H * H, lambda: LIN.linear_fwd(x, w, bias, "relu", out=y, ct=ct),
         lambda: torch.relu(torch.nn.functional.linear(x, w))),
        ("dgrad_hidden_nt", 2.0 * B * H * H, lambda: LIN.linear_dgrad_nt(x, wt, x, "relu", out=y, ct=ct),
         lambda: (x @ w) * (x > 0)),
        ("dgrad_hidden_bits", 2.0 * B * H * H,
         lambda: LIN.linear_dgrad_nt(x, wt, None, "relu", out=y, colpart=colpart, bits=bits),
         lambda: (x @ w) * (x > 0)),
        ("wgrad_hidden_nt", 2.0 * B * H * H, lambda: LIN.linear_wgrad_nt(xt, xt, out=gw),
         lambda: torch.matmul(x.t(), x, out=None).float()),
        ("transpose", 2.0 * B * H, lambda: LIN.transpose(x, out=xt), lambda: x.t().contiguous()),
        ("fwd_hidden", 2.0 * B * H * H, lambda: LIN.linear_fwd(x, w, bias, "relu", out=y),
         lambda: torch.relu(torch.nn.functional.linear(x, w))),
        ("dgrad_hidden", 2.0 * B * H * H, lambda: LIN.linear_dgrad(x, w, x, "relu", out=y),
         lambda: (x @ w) * (x > 0)),
        ("wgrad_hidden", 2.0 * B * H * H, lambda: LIN.linear_wgrad(x, x, out=gw),
         lambda: torch.matmul(x.t(), x, out=None).float()),
        ("fwd_in", 2.0 * B * 64 * H, lambda: LIN.linear_fwd(x64, w1, bias, "relu", out=y),
         lambda: torch.relu(torch.nn.functional.linear(x64, w1))),
        ("fwd_in_ct", 2.0 * B * 64 * H, lambda: LIN.linear_fwd(x64, w1, bias, "relu", out=y, ct=ct, bits=bits),
         lambda: torch.relu(torch.nn.functional.linear(x64, w1))),
        ("dgrad_out_ct", 2.0 * B * 64 * H,
         lambda: LIN.linear_dgrad_nt(x64, w1, None, "relu", out=y, ct=ct, colpart=colpart, bits=bits),
         lambda: (x64 @ w3) * (y > 0)),
        ("fwd_out", 2.0 * B * 64 * H, lambda: LIN.linear_fwd(x, w3, None, "none", torch.float32, out=y64),
         lambda: torch.nn.functional.linear(x, w3).float()),
        ("square_8192", 2.0 * 8192 ** 3, lambda: LIN.linear_fwd(x[:8192], w, None, "none", out=y[:8192]),
         lambda: torch.nn.functional.linear(x[:8192], w)),
    ]
    want = set(a.cases.split(",")) if a.cases else None
    for name, flop, ours, lib in cases:
        if want is not None and name not in want:
            continue
        t_o = timeit(ours, a.iters)
        t_l = timeit(lib, a.iters) if not a.no_lib else float("nan")
        print(json.dumps({"case": name, "B": B, "H": H, "ours_ms": round(t_o, 4), "lib_ms": round(t_l, 4),
                          "ours_tflops": round(flop / t_o / 1e9, 1), "lib_tflops": round(flop / t_l / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
