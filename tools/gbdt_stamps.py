#!/usr/bin/env python3
"""Phase stamps of the GBDT round kernels (block 0, last round of a reference-config fit).  Needs a
GBDT_STAMPS=1 build: `FILE=csrc/gbdt.hip bash tools/build_variant.sh gbdt_stamps -DGBDT_STAMPS=1`, then
`EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/gbdt_stamps.so python tools/gbdt_stamps.py`.
Prints one JSON line: per kernel, microseconds from its first stamp to each later phase, and each
kernel's start relative to the round's first histogram pass."""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from euromillioner_amd import config as C
    from euromillioner_amd.data.draws import DrawSet
    from euromillioner_amd.models.gbdt import GBDT
    from euromillioner_amd.ops import _native as N
    from euromillioner_amd.pipeline import gbdt_dataset

    ds = DrawSet.synthetic(n=None, seed=0, planted=0.5)
    X, Y, _ = gbdt_dataset(ds, C.RunConfig())
    m = int(0.7 * len(X))
    GBDT.from_params(C.RunConfig().gbdt_params(), nround=50, backend="hip").fit(X[:m], Y[:m], evals={"test": (X[m:], Y[m:])})
    buf = (ctypes.c_ulonglong * 512)()
    if N.lib().em_gbdt_stamps(buf) != 0:
        raise SystemExit("not a GBDT_STAMPS build")
    allst = np.array(buf[:], dtype=np.int64)
    st, clk = allst[:256], allst[256:]
    t0 = st[64]
    out = {}
    names = {0: "split0", 16: "split1", 32: "split2", 64: "hist0", 80: "hist1", 96: "hist2", 128: "update"}
    for base, name in names.items():
        seg = st[base:base + 16]
        if seg[0] == 0:
            continue
        out[name] = {"start_us": round((seg[0] - t0) / 100.0, 2),
                     "phases_us": [round((v - seg[0]) / 100.0, 2) if v else None for v in seg[1:8]]}
    # shader clock over the round (hist0 start -> update's first phase): cycles / (ticks / 100 MHz)
    if st[128] and st[64] and st[129]:
        out["shader_mhz"] = round(float(clk[129] - clk[64]) / ((st[129] - st[64]) / 100.0), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
