"""Plain-PyTorch losses / metrics: the fp32 reference the HIP kernels are tested against
and the CPU path of the framework.

``grouped_softmax_ce``: the 62 outputs are two categorical groups — 50 main numbers
and 12 stars — each trained with cross-entropy against the normalised multi-hot
target (5 ones / 5, 2 ones / 2).  ``bce``: independent sigmoids, mean over 62.

The reference has no neural loss at all (its learner is XGBoost ``reg:logistic`` with
``logloss``, ``/root/reference/src/main/java/com/euromillioner/Main.java:119,124``); these are
the DL4J-style heads of SURVEY.md §2.4 N5.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

MAIN = slice(0, 50)
STAR = slice(50, 62)


def grouped_softmax_ce(logits: torch.Tensor, target: torch.Tensor, reduction: str = "mean") -> torch.Tensor:
    z, y = logits[:, :62].float(), target[:, :62].float()
    lm = F.log_softmax(z[:, MAIN], dim=1)
    ls = F.log_softmax(z[:, STAR], dim=1)
    ym, ys = y[:, MAIN], y[:, STAR]
    nm = ym.sum(1, keepdim=True).clamp_min(1.0)
    ns = ys.sum(1, keepdim=True).clamp_min(1.0)
    per = -(ym * lm).sum(1) / nm.squeeze(1) - (ys * ls).sum(1) / ns.squeeze(1)
    return per.mean() if reduction == "mean" else (per.sum() if reduction == "sum" else per)


def bce(logits: torch.Tensor, target: torch.Tensor, reduction: str = "mean") -> torch.Tensor:
    per = F.binary_cross_entropy_with_logits(logits[:, :62].float(), target[:, :62].float(), reduction="none").mean(1)
    return per.mean() if reduction == "mean" else (per.sum() if reduction == "sum" else per)


LOSSES = {"softmax": grouped_softmax_ce, "bce": bce}


def draw_metrics_torch(logits: torch.Tensor, target: torch.Tensor, loss: str = "softmax") -> dict[str, float]:
    """Same definitions as the K13 kernel (csrc/metrics.hip), for CPU runs and tests."""
    z = logits[:, :62].float()
    y = target[:, :62].float() > 0.5
    n = z.shape[0]
    if n == 0:
        return {k: float("nan") for k in ("loss", "acc", "acc_thr", "hits_main", "hits_star", "exact", "trivial_acc")}
    top_m = torch.topk(z[:, MAIN], 5, dim=1).indices
    top_s = torch.topk(z[:, STAR], 2, dim=1).indices + 50
    pred = torch.zeros_like(y)
    pred.scatter_(1, top_m, True)
    pred.scatter_(1, top_s, True)
    if loss == "softmax":
        lp = torch.cat([F.log_softmax(z[:, MAIN], 1), F.log_softmax(z[:, STAR], 1)], 1)
        thr = lp >= -0.69314718
    else:
        thr = z >= 0
    mism = (pred ^ y).sum(1).float()
    mism_thr = (thr ^ y).sum(1).float()
    l = LOSSES[loss](logits, target, reduction="none")
    return {
        "loss": l.mean().item(),
        "acc": ((62 - mism) / 62).mean().item(),
        "acc_thr": ((62 - mism_thr) / 62).mean().item(),
        "hits_main": (pred[:, MAIN] & y[:, MAIN]).sum(1).float().mean().item(),
        "hits_star": (pred[:, STAR] & y[:, STAR]).sum(1).float().mean().item(),
        "exact": (mism == 0).float().mean().item(),
        "trivial_acc": ((62 - y.sum(1).float()) / 62).mean().item(),
    }
