#!/usr/bin/env python3
"""One large-GEMM case in a loop (for rocprofv3 PMC passes): python tools/gemm_one.py [--case fwd] [--iters 10]

fwd  : y[B,H] = x[B,H] @ w[H,H]^T (bf16 out, 256x256 NT path)
dgrad: dx[B,H] = dy[B,H] @ w[H,H] (via the transposed weight copy, NT)
sq   : M = N = K = H (fp32 out)
wgt  : dW[H,H] = dz^T x with transposed copies (fp32 out, K = B: the wide MLP's weight gradient)"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="fwd", choices=["fwd", "sq", "wgt"])
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--hidden", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from euromillioner_amd.ops import linear as LIN

    H = a.hidden
    if a.case == "wgt":
        g = torch.Generator(device="cuda").manual_seed(0)
        dzt = torch.rand(H, a.batch, device="cuda", generator=g).mul(2).sub(1).bfloat16()
        xt = torch.rand(H, a.batch, device="cuda", generator=g).mul(2).sub(1).bfloat16()
        out = torch.empty(H, H, device="cuda", dtype=torch.float32)
        run = lambda: LIN.linear_wgrad_nt(dzt, xt, out=out)  # noqa: E731
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        print(f"wgt M=N={H} K={a.batch}: {ms:.3f} ms  {2 * a.batch * H * H / ms / 1e9:.1f} TFLOP/s")
        return
    M = a.batch if a.case == "fwd" else H
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.rand(M, H, device="cuda", generator=g).mul(2).sub(1).bfloat16()
    w = torch.rand(H, H, device="cuda", generator=g).mul(2).sub(1).bfloat16()
    dt = torch.bfloat16 if a.case == "fwd" else torch.float32
    for _ in range(2):
        LIN.linear_fwd(x, w, None, "none", dt)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        LIN.linear_fwd(x, w, None, "none", dt)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    print(f"{a.case} M={M} N={H} K={H}: {ms:.3f} ms  {2 * M * H * H / ms / 1e9:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
