#!/usr/bin/env python3
"""Per-tile event trace of the v8 fused train kernel (csrc/mlp_fused.hip, EUROM_FUSED_V=8) in block 0:
when each forward wave started a tile, finished its softmax, and wrote + signalled it, and when each
backward wave saw it FULL and released it.  Needs a diagnostic side build (``FUSED_TRACE=1``, via
``tools/build_variant.sh trace -DFUSED_TRACE=1`` and EUROM_NATIVE_LIB); the shipped library records
nothing.  Prints the first tiles' timelines and the averages that say which side waited for which."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.ops import fused_mlp as FM

    B = int(os.environ.get("TR_B", 1 << 20))
    draws = generate_masks(B + 64, seed=1, planted=0.9)
    m = FusedSmallMLP("cuda", lr=1e-3)
    nslab = m.nslab_max
    K = (B // 32 + nslab - 1) // nslab
    ls = torch.zeros(nslab + K * 12 + 64, dtype=torch.float32, device="cuda")
    for _ in range(300):  # steady clocks
        FM.train_partials(draws, B, m.img, m.slabs, ls)
    torch.cuda.synchronize()
    FM.train_partials(draws, B, m.img, m.slabs, ls)
    torch.cuda.synchronize()
    raw = ls[nslab:nslab + K * 12].view(torch.int32).cpu().numpy().astype(np.int64).reshape(K, 12)
    wave = raw[:, 3].copy()
    t = raw & 0xFFFFFFFF
    t0 = t[0, 0]
    rel = (t - t0) & 0xFFFFFFFF
    rel = np.where(rel >= 1 << 31, rel - (1 << 32), rel).astype(np.float64) / 1e3  # k cycles
    start, comp, wrote = rel[:, 0], rel[:, 1], rel[:, 2]
    full = rel[:, 4:12:2]
    done = rel[:, 5:12:2]
    print(f"B={B}: {K} tiles in block 0; times in k cycles from tile 0's start")
    print("  k  wave  start  comp  wrote | B full seen (q0..q3)        | B done (q0..q3)")
    for k in range(min(K, int(os.environ.get("TR_ROWS", 40)))):
        print(f"{k:3d} {wave[k]:4d} {start[k]:6.1f} {comp[k]:5.1f} {wrote[k]:6.1f} | " +
              " ".join(f"{x:6.1f}" for x in full[k]) + " | " + " ".join(f"{x:6.1f}" for x in done[k]))
    fc = comp - start
    fw = wrote - comp
    lag = full.max(1) - wrote  # last backward wave's FULL seen after the write
    rd = done - full
    print(f"forward compute per tile: mean {fc.mean():.2f} med {np.median(fc):.2f} k; compute->written (slot wait + "
          f"writes): mean {fw.mean():.2f} med {np.median(fw):.2f} k")
    print(f"written -> last backward FULL seen: mean {lag.mean():.2f} med {np.median(lag):.2f} k; "
          f"backward read burst (FULL seen -> DONE): mean {rd.mean():.2f} k per wave")
    gaps = np.diff(done.max(1))
    print(f"consumption interval (tile k released by all 4): mean {gaps.mean():.2f} med {np.median(gaps):.2f} k; "
          f"production interval (sorted writes): med {np.median(np.diff(np.sort(wrote))):.2f} k")
    # ring occupancy when each tile is written: tiles written and not yet released by all 4
    rel_all = done.max(1)
    occ = [int(((wrote <= wrote[k]) & (rel_all > wrote[k])).sum()) for k in range(K)]
    print("ring occupancy at each write: mean %.2f, histogram %s" % (np.mean(occ), np.bincount(occ).tolist()))
    # what the backward side waited for: FULL seen - max(previous DONE, written)
    prev = np.concatenate([[0.0], done.max(1)[:-1]])
    bwait = full.min(1) - np.maximum(prev, 0)
    starved = (wrote > prev)
    print(f"backward starved (tile written after the previous tile's release) on {starved.mean() * 100:.0f} % of tiles; "
          f"mean gap previous release -> first FULL seen {bwait.mean():.2f} k")
    print("per forward wave: tiles", np.bincount(wave, minlength=8).tolist(), "mean compute",
          [round(float(fc[wave == w].mean()), 2) for w in range(8)])


if __name__ == "__main__":
    main()
