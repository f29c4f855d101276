#!/usr/bin/env python3
"""Where the wall time of the GBDT reference fit goes on the host (cProfile of a warm fit), and the fit
time against `rounds_per_call` (the host reads the metric history back after every call)."""
from __future__ import annotations

import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from euromillioner_amd import config as C
    from euromillioner_amd.data.draws import DrawSet
    from euromillioner_amd.models import gbdt_hip as GH
    from euromillioner_amd.models.gbdt import GBDT
    from euromillioner_amd.pipeline import gbdt_dataset

    cfg = C.RunConfig()
    ds = DrawSet.synthetic(n=None, seed=0, planted=0.5)
    X, Y, _ = gbdt_dataset(ds, cfg)
    m = int(0.7 * len(X))
    ev = {"test": (X[m:], Y[m:])}
    GBDT.from_params(cfg.gbdt_params(), nround=2, backend="hip").fit(X[:m], Y[:m], evals=ev)
    orig = GH.fit
    for rpc in (100, 500):
        GH.fit = lambda *a, rpc=rpc, **k: orig(*a, rounds_per_call=rpc, **k)
        best = float("inf")
        for _ in range(3):
            g = GBDT.from_params(cfg.gbdt_params(), nround=500, backend="hip")
            t0 = time.perf_counter()
            g.fit(X[:m], Y[:m], evals=ev)
            best = min(best, time.perf_counter() - t0)
        print(json.dumps({"rounds_per_call": rpc, "fit_s": round(best, 4)}), flush=True)
    GH.fit = orig
    g = GBDT.from_params(cfg.gbdt_params(), nround=500, backend="hip")
    pr = cProfile.Profile()
    pr.enable()
    g.fit(X[:m], Y[:m], evals=ev)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(25)
    print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
