"""Evaluation metrics (T7).

* :func:`check_predicts` — output-compatible port of ``Main.checkPredicts``
  (``Main.java:150-162``): true iff both prediction matrices have the same number of
  rows and every row is bit-for-bit equal (``Arrays.equals`` on float[]).  Kept for
  parity; it is not an accuracy metric (defect D-e).
* :func:`logloss` — XGBoost's ``eval_metric=logloss`` (``Main.java:124``), with the
  same clipping of probabilities to [1e-16, 1 - 1e-16].
* :func:`draw_metrics` — the metrics that make the README's "0.9+" (``README.md:5``)
  meaningful for 62-wide draw vectors: element-wise accuracy of the structured
  (top-5 + top-2) prediction next to its all-zero trivial floor (55/62 = 0.887), the
  thresholded accuracy, hit rates and exact-draw matches.  Same definitions as the
  GPU kernel in ``csrc/metrics.hip``.
"""
from __future__ import annotations

import numpy as np

TRIVIAL_ACC = 55.0 / 62.0


def check_predicts(f_predicts, s_predicts) -> bool:
    if len(f_predicts) != len(s_predicts):
        return False
    for a, b in zip(f_predicts, s_predicts):
        a = np.asarray(a, dtype=np.float32).reshape(-1)
        b = np.asarray(b, dtype=np.float32).reshape(-1)
        # Arrays.equals(float[], float[]) compares floatToIntBits: NaN == NaN, +0 != -0
        if a.shape != b.shape or not np.array_equal(a.view(np.int32), b.view(np.int32)):
            return False
    return True


def logloss(y: np.ndarray, p: np.ndarray, eps: float = 1e-16) -> float:
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    p = np.clip(np.asarray(p, dtype=np.float64).reshape(-1), eps, 1.0 - eps)
    if y.size == 0:
        return float("nan")
    return float(-np.mean(y * np.log(p) + (1.0 - y) * np.log(1.0 - p)))


def rmse(y: np.ndarray, p: np.ndarray) -> float:
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    p = np.asarray(p, dtype=np.float64).reshape(-1)
    return float(np.sqrt(np.mean((y - p) ** 2))) if y.size else float("nan")


def error_rate(y: np.ndarray, p: np.ndarray) -> float:
    """XGBoost ``error``: fraction with (p > 0.5) != y."""
    y = np.asarray(y).reshape(-1)
    p = np.asarray(p).reshape(-1)
    return float(np.mean((p > 0.5).astype(np.float64) != y)) if y.size else float("nan")


def mlogloss(y: np.ndarray, p: np.ndarray, eps: float = 1e-16) -> float:
    """XGBoost ``mlogloss``: y one-hot (or class ids) [n, K], p class probabilities [n, K]."""
    p = np.asarray(p, dtype=np.float64)
    y = np.asarray(y)
    lab = y.reshape(-1).astype(np.int64) if y.ndim == 1 else np.argmax(y, axis=1)
    if p.shape[0] == 0:
        return float("nan")
    return float(-np.mean(np.log(np.maximum(p[np.arange(len(p)), lab], eps))))


def merror(y: np.ndarray, p: np.ndarray) -> float:
    """XGBoost ``merror``: fraction of rows whose arg-max class is wrong."""
    p = np.asarray(p)
    y = np.asarray(y)
    lab = y.reshape(-1).astype(np.int64) if y.ndim == 1 else np.argmax(y, axis=1)
    return float(np.mean(np.argmax(p, axis=1) != lab)) if len(p) else float("nan")


EVAL_METRICS = {"logloss": logloss, "rmse": rmse, "error": error_rate, "mlogloss": mlogloss, "merror": merror}


def _topk_mask(z: np.ndarray, k: int) -> np.ndarray:
    # stable: earlier index wins ties (matches the kernel's insertion order)
    idx = np.argsort(-z, axis=1, kind="stable")[:, :k]
    m = np.zeros_like(z, dtype=bool)
    np.put_along_axis(m, idx, True, axis=1)
    return m


def draw_metrics(scores: np.ndarray, target: np.ndarray, loss: str = "softmax") -> dict:
    """scores: [N, 62] logits; target: [N, 62] multi-hot."""
    z = np.asarray(scores, dtype=np.float64)[:, :62]
    y = np.asarray(target)[:, :62] > 0.5
    n = len(z)
    if n == 0:
        return {}
    pred = np.concatenate([_topk_mask(z[:, :50], 5), _topk_mask(z[:, 50:], 2)], axis=1)
    if loss == "softmax":
        def lsm(a):
            m = a.max(1, keepdims=True)
            return a - m - np.log(np.exp(a - m).sum(1, keepdims=True))

        lp = np.concatenate([lsm(z[:, :50]), lsm(z[:, 50:])], axis=1)
        thr = lp >= np.log(0.5)
        nm = np.maximum(y[:, :50].sum(1), 1)
        ns = np.maximum(y[:, 50:].sum(1), 1)
        lossv = -(lp[:, :50] * y[:, :50]).sum(1) / nm - (lp[:, 50:] * y[:, 50:]).sum(1) / ns
    else:
        thr = z >= 0
        lossv = (np.maximum(z, 0) + np.log1p(np.exp(-np.abs(z))) - y * z).mean(1)
    mism = (pred ^ y).sum(1)
    return {
        "loss": float(lossv.mean()),
        "acc": float(((62 - mism) / 62).mean()),
        "acc_thr": float(((62 - (thr ^ y).sum(1)) / 62).mean()),
        "hits_main": float((pred[:, :50] & y[:, :50]).sum(1).mean()),
        "hits_star": float((pred[:, 50:] & y[:, 50:]).sum(1).mean()),
        "exact": float((mism == 0).mean()),
        "trivial_acc": float(((62 - y.sum(1)) / 62).mean()),
        "count": int(n),
    }


def chance_levels() -> dict:
    """Expected metrics of a uniformly random structured prediction on iid draws."""
    hm, hs = 5 * 5 / 50, 2 * 2 / 12
    return {"hits_main": hm, "hits_star": hs, "acc": (62 - 2 * (5 - hm) - 2 * (2 - hs)) / 62,
            "trivial_acc": TRIVIAL_ACC}
