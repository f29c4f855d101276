#!/usr/bin/env python3
"""GBDT engine benchmark: the reference configuration (Main.java:113-138: gbtree, eta 1, depth 3,
gamma 1, reg:logistic, logloss watch, 500 rounds) on the reference-sized draw history
(~1.33k draws, 62 next-draw boosters), HIP engine vs the numpy oracle, plus a large synthetic
draw set to show device throughput.  One JSON line per case."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from euromillioner_amd import config as C
    from euromillioner_amd.data.draws import DrawSet
    from euromillioner_amd.models.gbdt import GBDT
    from euromillioner_amd.pipeline import gbdt_dataset

    cfg = C.RunConfig()
    cases = [("reference_calendar", None, 500, True), ("synthetic_262k", 262145, 50, False)]
    only = sys.argv[1] if len(sys.argv) > 1 else None
    hip_only = only == "hip"  # every case, HIP engine only
    if hip_only:
        only = None
    for name, n, rounds, with_numpy in cases:
        if only and only not in name:
            continue
        ds = DrawSet.synthetic(n=n, seed=0, planted=0.5)
        X, Y, _ = gbdt_dataset(ds, cfg)
        m = int(0.7 * len(X))
        res = {"case": name, "rows": m, "features": X.shape[1], "tasks": Y.shape[1], "rounds": rounds}
        runs = [("hip", "auto")]
        if n is not None:  # large case: the exact fp64 histogram form too (auto = fixed point here)
            runs.append(("hip", "exact"))
        if with_numpy and not only and not hip_only:
            runs.append(("numpy", "auto"))
        for be, mode in runs:
            if be == "hip":  # exclude one-time GPU context / code-object load from the timing
                GBDT.from_params(cfg.gbdt_params(), nround=2, backend=be, hist_mode=mode).fit(
                    X[:m], Y[:m], evals={"test": (X[m:], Y[m:])})
            dt = float("inf")
            for _ in range(2 if be == "hip" else 1):  # best of two: the first fit of a mode may run on a cold clock
                g = GBDT.from_params(cfg.gbdt_params(), nround=rounds, backend=be, hist_mode=mode)
                t0 = time.perf_counter()
                g.fit(X[:m], Y[:m], evals={"test": (X[m:], Y[m:])})
                dt = min(dt, time.perf_counter() - t0)
            key = be if mode == "auto" else f"{be}_{mode}"
            res[f"{key}_s"] = round(dt, 3)
            res[f"{key}_test_logloss"] = g.history[-1]["test"]
            res[f"{key}_trees_per_s"] = round(rounds * Y.shape[1] / dt, 1)
            res[f"{key}_quant_bits"] = int(getattr(g, "quant_bits_used", 0))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
