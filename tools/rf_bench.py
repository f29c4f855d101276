#!/usr/bin/env python3
"""Random-forest benchmark (BASELINE config 4: 100 trees over 62 one-hot features, 1xMI355X).

    python tools/rf_bench.py [--rows 1000000] [--trees 100] [--depth 8] [--repeat 3]

Times the full GPU fit (bootstrap, all levels of all trees, node records) and the batched
predict, plus validation metrics; prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--trees", type=int, default=100)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--subset", default="sqrt")
    ap.add_argument("--planted", type=float, default=0.9)
    ap.add_argument("--repeat", type=int, default=3)
    a = ap.parse_args()
    from euromillioner_amd.data.synthetic import generate_draws
    from euromillioner_amd.data.draws import mask_bits
    from euromillioner_amd.models.forest import RandomForest, n_candidates
    from euromillioner_amd.ops import forest as K
    from euromillioner_amd.ops import fused_mlp as FM

    nums, _ = generate_draws(a.rows + 1, seed=0, planted=a.planted, native=True)
    m = mask_bits(nums)
    n_tr = int(0.7 * a.rows)
    dev = torch.device("cuda")
    md = torch.from_numpy(m.view(np.int64)).to(dev)
    Xtr, Ytr = md[:n_tr].reshape(-1, 1).contiguous(), md[1:n_tr + 1].contiguous()
    k = n_candidates(a.subset, 62)
    K.fit(Xtr[:1000], Ytr[:1000], 62, 0, 2, 3, k, 1, True, 0)  # warm-up / load
    torch.cuda.synchronize()
    times = []
    for _ in range(a.repeat):
        t0 = time.perf_counter()
        feat, value, gain, cover = K.fit(Xtr, Ytr, 62, 0, a.trees, a.depth, k, 1, True, 0, return_device=True)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    n_val = a.rows - n_tr
    Xv = md[n_tr:a.rows].reshape(-1, 1).contiguous()
    pred_times = []
    for _ in range(1 + a.repeat):  # the first call pays one-time costs (code object load, LDS attribute)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lg = K.predict(Xv, feat, value, a.depth, out_logit=True)
        torch.cuda.synchronize()
        pred_times.append(time.perf_counter() - t0)
    t_pred = min(pred_times[1:]) if len(pred_times) > 1 else pred_times[0]
    part = FM.draw_metrics(lg, md, n_val, loss="bce", offset=n_tr).double().sum(0).cpu().numpy()
    cnt = part[7]
    val = {kk: float(part[i] / cnt) for i, kk in enumerate(FM.METRIC_NAMES[:-1])}
    fit_s = min(times)
    print(json.dumps({"metric": "random forest fit (100 trees, 62 one-hot features)", "rows": n_tr,
                      "trees": a.trees, "max_depth": a.depth, "k_features": k, "fit_s": fit_s,
                      "fit_rows_x_trees_per_s": n_tr * a.trees / fit_s, "predict_s": t_pred, "predict_first_call_s": pred_times[0],
                      "predict_rows_per_s": n_val / t_pred, "nodes_split": int((feat >= 0).sum().item()),
                      "val": val}))


if __name__ == "__main__":
    main()
