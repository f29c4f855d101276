#!/usr/bin/env python3
"""Where a pp16 GEMM K-tile's time goes, from the diagnostic segment timers (G_STAMPS build).

build:  python -m euromillioner_amd._build --define G_STAMPS=1 ; cp the lib to euromillioner_amd/lib/ab/stamps.so ;
        rebuild without --define.   run:  EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/stamps.so python tools/gemm_stamps.py
Prints, per wave group (G0 = waves 0-3, G1 = 4-7), the mean cycles per segment of each timer
(see csrc/gemm.hip G_STAMPS) and per dispatch the prologue / epilogue cycles."""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ["ld_issue", "ld_vmcnt", "ld_barrier", "mf_lgkm", "mf_issue", "mf_barrier", "prologue", "epilogue"]


def main():
    from euromillioner_amd.ops import _native as N
    from euromillioner_amd.ops import linear as LIN

    N.register_signatures({"em_gemm_stamps": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_int64])})
    M, NN, K = (int(v) for v in os.environ.get("STAMP_SHAPE", "65536,8192,8192").split(","))
    ct = os.environ.get("STAMP_CT", "0") == "1"
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(NN, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.zeros(NN, device="cuda")
    y = torch.empty(M, NN, dtype=torch.bfloat16, device="cuda")
    cbuf = torch.empty(NN, M, dtype=torch.bfloat16, device="cuda") if ct else None
    for _ in range(5):
        LIN.linear_fwd(x, w, b, "relu", out=y, ct=cbuf)
    torch.cuda.synchronize()
    nblk = 4096
    host = np.zeros(nblk * 8 * 8, dtype=np.uint64)
    N.call("em_gemm_stamps", host.ctypes.data, host.nbytes)
    tiles = (M // 256) * (NN // 256)
    nb = min(nblk, tiles)
    a = host.reshape(nblk, 8, 8)[:nb].astype(np.float64)
    segs = 4 * (K // 64)  # load + MFMA segments per wave
    out = {"shape": [M, NN, K], "ct": ct, "blocks": nb}
    for gi, sl in (("G0", slice(0, 4)), ("G1", slice(4, 8))):
        m = a[:, sl, :].mean(axis=(0, 1))
        out[gi] = {n: round(float(m[i] / (segs if i < 6 else 1)), 1) for i, n in enumerate(NAMES)}
    per_slot = sum(out["G0"][n] for n in NAMES[:6]) / 2  # a wave spends 2 slots per phase (load + MFMA)
    out["slot_cycles"] = round(per_slot, 1)
    out["mfma_issue_share"] = round(out["G0"]["mf_issue"] / per_slot, 3)
    # per block: the K loop's segments + prologue + epilogue; the fixed share is what a persistent kernel
    # overlapping a tile's epilogue with the next tile's first K-tiles could hide at most
    loop = segs * sum(out["G0"][n] for n in NAMES[:6]) / 2
    blk = loop + out["G0"]["prologue"] + out["G0"]["epilogue"]
    out["block_cycles"] = round(blk, 1)
    out["fixed_share"] = round((out["G0"]["prologue"] + out["G0"]["epilogue"]) / blk, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
