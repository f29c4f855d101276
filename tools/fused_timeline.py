#!/usr/bin/env python3
"""Per-block wall-clock timeline of the fused train kernel (csrc/mlp_fused.hip) inside a 10-launch
hipGraph (steady clock).  Needs a diagnostic build: ``python -m euromillioner_amd._build --define
FUSED_STAMPS=1`` into a side library (EUROM_NATIVE_LIB), never the shipped one -- the stamps drain LDS
counters at every mark.  Prints, per batch size, the spread of block entry, prologue, loop and slab-write
times of the LAST launch of the graph, the per-XCD-group loop medians and the forward / backward wave
phase split (s_memtime cycles, ``Stamps`` marks 0-9)."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ["F wait slot", "F X+F1+H", "F F2", "F loss", "F D2+signal",
         "B wait full", "B reads", "B B1+dW2+db2", "B mask", "B dW1T"]



def main():
    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.ops import fused_mlp as FM

    draws = generate_masks((1 << 23) + 16, seed=1, planted=0.9)
    m = FusedSmallMLP("cuda", lr=1e-3)
    for B in [int(x) for x in os.environ.get("TL_B", "262144,1048576,2097152,4194304").split(",")]:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            nslab = FM.train_partials(draws, B, m.img, m.slabs, m.loss_slabs, loss="softmax")
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(10):
                    FM.train_partials(draws, B, m.img, m.slabs, m.loss_slabs, loss="softmax")
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(30):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        per = e0.elapsed_time(e1) * 1e3 / 10
        v8 = os.environ.get("EUROM_FUSED_V") in ("8", "9")  # v8 / v9: 12 waves, wall-clock marks in wave 0's spare lanes 10-14
        T0 = FM.P_TOTAL + (10 if v8 else 128)
        raw = m.slabs[:nslab, T0:T0 + 4].contiguous().view(torch.int32).cpu().numpy()
        t = raw.astype(np.int64) & 0xFFFFFFFF
        t -= t[:, 0].min()
        us = t / 100.0
        loop = us[:, 2] - us[:, 1]
        q = lambda a: "min %.1f med %.1f max %.1f" % (a.min(), np.median(a), a.max())
        print(f"B={B}: {per:.1f} us/launch (graph); entry spread {us[:, 0].max():.2f}; prologue {q(us[:, 1] - us[:, 0])};"
              f" loop {q(loop)}; fold {q(us[:, 3] - us[:, 2])}; first entry -> last fold {us[:, 3].max():.1f}", flush=True)
        xcd = np.arange(nslab) % 8
        print("   loop median per blockIdx%8:", " ".join("%.1f" % np.median(loop[xcd == k]) for k in range(8)))
        # which physical XCD ran each block (s_getreg HW_REG_XCC_ID): is the slow group a fixed XCD
        # across launches, or a fixed blockIdx % 8?  Five more single launches.
        for rep in range(5):
            torch.cuda.synchronize()
            with torch.cuda.stream(s):
                FM.train_partials(draws, B, m.img, m.slabs, m.loss_slabs, loss="softmax")
            torch.cuda.synchronize()
            raw = m.slabs[:nslab, T0:T0 + 5].contiguous().view(torch.int32).cpu().numpy()
            t = raw[:, :4].astype(np.int64) & 0xFFFFFFFF
            lp = (t[:, 2] - t[:, 1]) / 100.0
            xc = raw[:, 4]
            print(f"   launch {rep}: loop median per XCC_ID:",
                  " ".join("%d:%.1f" % (k, np.median(lp[xc == k])) for k in range(8) if (xc == k).any()),
                  "| blockIdx%8 -> XCC_ID:", " ".join(str(int(np.bincount(xc[xcd == k]).argmax())) for k in range(8)))
        nw = 12 if v8 else 8
        st = m.slabs[:nslab, FM.P_TOTAL:FM.P_TOTAL + 16 * nw].reshape(nslab, nw, 16)[:, :, :10].double().cpu().numpy()
        shared = os.environ.get("TL_SHARED", "1") == "1"  # FUSED_SHARED layout: waves 0-3 forward
        if v8:
            roles = (("forward", list(range(8))), ("backward", [8, 9, 10, 11]))
        else:
            roles = (("forward", [0, 1, 2, 3]), ("backward", [4, 5, 6, 7])) if shared else \
                (("forward", [0, 1, 6, 7]), ("backward", [2, 3, 4, 5]))
        for nm, ws in roles:  # wave -> role map of the kernel
            v = st[:, ws, :].reshape(-1, 10).mean(0)
            tot = v.sum()
            print(f"   {nm}: {tot / 1e3:.1f} k cycles/wave; " +
                  ", ".join(f"{n} {x / 1e3:.1f}k" for n, x in zip(NAMES, v) if x > 0))
            # per wave slot: total / waiting (phase 0 forward, 5 backward), medians over blocks
            wi = 0 if nm == "forward" else 5
            print("      per wave (total/wait k):", " ".join(
                "w%d %.0f/%.0f" % (w, np.median(st[:, w, :].sum(1)) / 1e3, np.median(st[:, w, wi]) / 1e3) for w in ws))


if __name__ == "__main__":
    main()
