"""End-to-end pipelines (T8).

:func:`run_reference_pipeline` is the MI355X-native counterpart of ``Main.main``
(``Main.java:35-148``): acquire draws -> featurize -> positional 70/30 split ->
XGBoost-semantics GBDT (500 rounds, the reference's parameter map) with a train/test
watch list -> predict -> print ``checkPredicts`` -> plus a metrics JSON line.

Differences from the reference, all documented in SURVEY.md §7.5:
* acquisition: no network — synthetic draws on the reference's calendar, a CSV, or an
  offline copy of the HTML page (``--html``);
* CSVs are proper newline-terminated files written to ``--workdir`` (D-b/D-c/D-h);
* default target is the next draw (62 boosters), because the reference's label
  (column 0 = day_of_week, 1..7) is invalid for ``reg:logistic`` (D-d); ``--target
  reference`` reproduces it (and fails the same way XGBoost does unless the objective
  is changed, e.g. ``--objective reg:squarederror``);
* ``--reference-compat`` reproduces D-f (a second booster trained on the validation
  split) so ``check_predicts`` compares the same two arrays as the reference;
* errors are reported accurately with a non-zero exit code (D-g).
"""
from __future__ import annotations

import datetime as _dt
import os
import tempfile
import time

import numpy as np

from . import log as L
from . import metrics as M
from .config import RunConfig
from .data.draws import DrawSet, featurize_raw, multi_hot, positional_split


def load_draws(cfg: RunConfig) -> DrawSet:
    d = cfg.data
    if d.source == "device":
        raise ValueError("data.source=device (GPU-generated, HBM-resident draws) feeds MLP training only")
    if d.source == "synthetic":
        ds = DrawSet.synthetic(n=d.n_draws, seed=d.seed, planted=d.planted)
    elif d.source == "csv":
        from .data.csv_io import read_draws_csv

        hdr = {"auto": None, "yes": True, "no": False}.get(str(d.header).lower())
        if hdr is None and str(d.header).lower() != "auto":
            raise ValueError("--header must be auto, yes or no")
        ds = read_draws_csv(_need(d.path), header=hdr)
    elif d.source == "reference-csv":
        from .data.csv_io import read_reference_csv, reference_records_to_drawset

        paths = [p for p in _need(d.path).split(",") if p]
        ds = reference_records_to_drawset(np.concatenate([read_reference_csv(p) for p in paths]))
    elif d.source == "html":
        from .data.html_table import parse_results_table

        with open(_need(d.path), encoding="utf-8") as f:
            ds = parse_results_table(f.read(), d.html_table_class)
    else:
        raise ValueError(f"unknown data source {d.source!r}")
    if ds.dates is not None and len(ds):
        lo = np.datetime64(d.from_date, "D")
        hi = np.datetime64(d.to_date, "D")
        keep = (ds.dates >= lo) & (ds.dates <= hi)
        if not keep.all() and d.source != "synthetic":
            ds = DrawSet(ds.numbers[keep], ds.dates[keep], ds.meta)
    ds.validate()
    return ds


def _need(path):
    if not path:
        raise ValueError("this data source needs --data-path")
    if not os.path.exists(path.split(",")[0]):
        raise FileNotFoundError(path)
    return path


def gbdt_dataset(ds: DrawSet, cfg: RunConfig):
    """(X, Y, feature names) for the configured GBDT target."""
    if cfg.gbdt.target == "reference":
        raw = featurize_raw(ds).astype(np.float64)
        lc = cfg.data.label_column
        y = raw[:, lc]
        X = np.delete(raw, lc, axis=1)
        return X, y[:, None], "reference"
    # next-draw: multi-hot of draw t (+ its date fields) -> multi-hot of draw t+1, 62 boosters
    X = multi_hot(ds.numbers[:-1]).astype(np.float64)
    if ds.dates is not None:
        raw = featurize_raw(ds)[:-1, :4].astype(np.float64)
        X = np.concatenate([X, raw], axis=1)
    Y = multi_hot(ds.numbers[1:]).astype(np.float64)
    return X, Y, "next-draw"


def run_reference_pipeline(cfg: RunConfig, out=None) -> dict:
    log = L.get("Main")
    t0 = time.time()
    ds = load_draws(cfg)
    log.info(f"loaded {len(ds)} draws from {cfg.data.source} "
             f"({ds.meta.get('planted', 0.0) if cfg.data.source == 'synthetic' else 'n/a'} planted)")
    tmp = None
    if cfg.data.workdir:
        workdir = cfg.data.workdir
        os.makedirs(workdir, exist_ok=True)
    else:  # D-h: the reference leaks its temp CSVs; ours are removed when the run ends
        tmp = tempfile.TemporaryDirectory(prefix="emn_")
        workdir = tmp.name
    X, Y, target = gbdt_dataset(ds, cfg)
    n = len(X)
    margin = positional_split(n, cfg.data.train_pct)
    Xtr, Ytr, Xva, Yva = X[:margin], Y[:margin], X[margin:], Y[margin:]
    # materialise the split like Main.java:69-108 (fixed format), for inspection / reuse
    from .data.csv_io import write_draws_csv

    write_draws_csv(os.path.join(workdir, "emn.csv"), ds.slice(0, margin + (1 if target == "next-draw" else 0)))
    write_draws_csv(os.path.join(workdir, "emn_validation.csv"), ds.slice(margin, len(ds)))

    from .models.gbdt import GBDT

    g = cfg.gbdt
    mk = dict(nround=g.nround, reg_lambda=g.reg_lambda, min_child_weight=g.min_child_weight,
              base_score=g.base_score, max_bin=g.max_bin, backend=_gbdt_backend(cfg), log=log,
              log_every=max(1, g.nround // 20))
    # data-parallel boosting (C4) under torchrun: row shards, all-reduced histograms, identical trees
    from .parallel import dist as D

    info = D.init(cfg.dist.backend, cfg.dist.timeout_s, device="cpu" if _gbdt_backend(cfg) == "numpy" else cfg.device)
    group = info.group if info.is_dist else None
    a, b = D.shard_range(len(Xtr), info)
    va, vb = D.shard_range(len(Xva), info)
    watches = {"train": (Xtr[a:b], Ytr[a:b]), "test": (Xva[va:vb], Yva[va:vb])}
    booster = GBDT.from_params(cfg.gbdt_params(), **mk).fit(Xtr[a:b], Ytr[a:b], evals=watches, group=group)
    p_train = booster.predict(Xtr)
    if cfg.reference_compat:
        booster_test = GBDT.from_params(cfg.gbdt_params(), **mk).fit(Xva[va:vb], Yva[va:vb], evals=watches,
                                                                      group=group)  # D-f
        p_val = booster_test.predict(Xva)
    else:
        p_val = booster.predict(Xva)
    compat = M.check_predicts(p_train, p_val)
    if info.rank == 0:
        (out.write if out else print)(str(compat).lower() + ("\n" if out else ""))  # Main.java:143 prints the boolean
    res = {"pipeline": "reference", "target": target, "n_draws": len(ds), "n_train": int(margin),
           "n_val": int(n - margin), "backend": booster.backend_used, "check_predicts": compat,
           "train_" + booster.eval_metric: booster.history[-1].get("train") if booster.history else None,
           "val_" + booster.eval_metric: booster.history[-1].get("test") if booster.history else None,
           "seconds": round(time.time() - t0, 3), "workdir": workdir}
    if target == "next-draw" and len(Xva):
        margins = booster.predict_margin(Xva)
        res["val"] = M.draw_metrics(margins, Yva, loss="bce")
        res["chance"] = M.chance_levels()
    res["world_size"] = info.world
    if cfg.ckpt.path and info.rank == 0:
        booster.save(cfg.ckpt.path)
        res["checkpoint"] = cfg.ckpt.path
    D.shutdown(info)
    if tmp is not None:
        tmp.cleanup()
        res["workdir"] = None
    return res


def _gbdt_backend(cfg: RunConfig) -> str:
    dev = cfg.gbdt.device if cfg.gbdt.device != "auto" else cfg.device
    if dev == "cpu":
        return "numpy"
    if dev == "cuda":
        return "hip"
    return "auto"


def date_str(d) -> str:
    return str(np.datetime64(d, "D")) if d is not None else ""


def next_draw_date(last: np.datetime64) -> np.datetime64:
    """The next Euromillions draw day after ``last`` (Fridays; Tuesdays too from 2011-05-10).  Pure
    datetime64 arithmetic: long synthetic sequences run past year 9999, where datetime.date cannot go."""
    tuesdays_from = np.datetime64("2011-05-10", "D")
    d = np.datetime64(last, "D") + np.timedelta64(1, "D")
    while True:
        wd = (int(d.astype(np.int64)) + 3) % 7  # 1970-01-01 was a Thursday; Monday = 0 as in date.weekday()
        if wd == 4 or (wd == 1 and d >= tuesdays_from):
            return d
        d = d + np.timedelta64(1, "D")
