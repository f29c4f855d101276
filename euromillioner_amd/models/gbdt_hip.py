"""Device side of :mod:`euromillioner_amd.models.gbdt`: buffers + calls into ``csrc/gbdt.hip``.

Replaces the reference's ``XGBoost.train`` / ``Booster.predict`` JNI calls
(``/root/reference/src/main/java/com/euromillioner/Main.java:136-141``):
all rounds and levels run on the stream from the native driver ``em_gbdt_fit``; under data
parallelism (C4) the per-level histogram is all-reduced between the hist and split kernels."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ..ops import _native as N
from .gbdt import TreeArrays, apply_bins, quant_bits

_v, _i, _i64, _f, _u32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_uint32


class _Eval(ctypes.Structure):
    _fields_ = [("bins", _v), ("Y", _v), ("margin", _v), ("n", _i)]


N.register_signatures({
    "em_gbdt_fit": (_i, [_v, _v, _i, _i, _v, _v, _i, _v, ctypes.POINTER(_Eval), _i, _i, _i, _i, _i, _i, _f, _f, _f,
                         _f, _f, _u32, _v, _v, _v, _v, _v, _i64, _v, _v, _v, _v, _v, _v, _v, _v, _v, _v, _i, _i, _v]),
    "em_gbdt_partial_doubles": (_i64, [_i, _i, _i, _v, _i]),
    "em_gbdt_fused_error": (_i, []),
    "em_gbdt_init_margin": (_i, [_v, _i64, _f, _v]),
    "em_gbdt_predict": (_i, [_v, _v, _i, _i, _i, _i, _i, _i, _v, _v, _v, _v, _v]),
    "em_gbdt_dp_round_begin": (_i, [_i, _i, _i, _i, _v, _v, _v, _v, _v, _i, _f, _u32, _v, _v, _v, _v, _v]),
    "em_gbdt_dp_level_hist": (_i, [_i, _v, _v, _v, _v, _i, _i, _i, _v, _v, _v, _i64, ctypes.POINTER(_i64), _v]),
    "em_gbdt_dp_level_split": (_i, [_i, _v, _v, _i, _i, _i, _v, _i, _i, _v, _v, _v, _v, _v, _v, _v, _f, _f, _v]),
    "em_gbdt_dp_round_end": (_i, [_i, _i, _i, _v, _v, _v, _v, _v, _v, _v, _v, _v, _f, _f, _f, _v]),
    "em_gbdt_metric_sum": (_i, [_v, _v, _i, _i, _i, _i, _v, _v, _v]),
})

OBJ = {"reg:logistic": 0, "binary:logistic": 0, "reg:squarederror": 1, "multi:softprob": 2, "multi:softmax": 2}
MET = {"logloss": 0, "rmse": 1, "error": 2, "mlogloss": 3, "merror": 4}


def _dev():
    return torch.device("cuda", torch.cuda.current_device())


class PlanUnsupported(ValueError):
    """The device engine has no histogram plan for this shape (per-level histograms too large)."""


class _Cells:
    """Compact histogram axis: feature f owns bins [off[f], off[f+1]) (host array for the native
    tile planner, device copy for the kernels)."""

    def __init__(self, cuts, dev):
        nbf = np.array([len(c) + 1 for c in cuts], dtype=np.int64)
        if (nbf > 256).any():
            raise PlanUnsupported("GPU GBDT supports at most 256 bins per feature")
        self.host = np.ascontiguousarray(np.concatenate([[0], np.cumsum(nbf)]).astype(np.int32))
        self.dev = torch.from_numpy(self.host).to(dev)
        self.C = int(self.host[-1])

    @property
    def hp(self):
        return self.host.ctypes.data


def fit(model, X, bins, nbins, Y, evals, rounds_per_call: int = 500, dp=None):
    dev = _dev()
    n, F = bins.shape
    T = Y.shape[1]
    R, D = model.nround, model.max_depth
    NN = 2 ** (D + 1) - 1
    cells = _Cells(model.cuts, dev)
    d_bins = torch.from_numpy(np.ascontiguousarray(bins, dtype=np.uint8)).to(dev)
    d_Y = torch.from_numpy(np.ascontiguousarray(Y, dtype=np.float32)).to(dev)
    margin = torch.empty(T * n, dtype=torch.float32, device=dev)
    stream = N.stream_handle(dev)
    N.call("em_gbdt_init_margin", margin.data_ptr(), T * n, float(model.base_margin), stream)
    ev_names = list(evals.keys())
    ev_keep = []
    ev_structs = (_Eval * max(1, len(ev_names)))()
    for i, name in enumerate(ev_names):
        ex, ey = evals[name]
        eb = apply_bins(np.asarray(ex, np.float64), model.cuts)
        db = torch.from_numpy(np.ascontiguousarray(eb, dtype=np.uint8)).to(dev)
        dy = torch.from_numpy(np.ascontiguousarray(np.asarray(ey, np.float32).reshape(len(ex), -1))).to(dev)
        em = torch.empty(T * len(ex), dtype=torch.float32, device=dev)
        N.call("em_gbdt_init_margin", em.data_ptr(), em.numel(), float(model.base_margin), stream)
        ev_keep += [db, dy, em]
        ev_structs[i] = _Eval(db.data_ptr(), dy.data_ptr(), em.data_ptr(), len(ex))
    g = torch.empty(T * n, dtype=torch.float32, device=dev)
    h = torch.empty_like(g)
    node = torch.empty(T * n, dtype=torch.int16, device=dev)
    node2 = torch.empty_like(node)  # the fused round's double-buffered level nodes
    pdoubles = N.query("em_gbdt_partial_doubles", n, T, F, cells.hp, D)
    if pdoubles < 0:
        raise PlanUnsupported(f"GPU GBDT: no histogram plan for depth {D} x {cells.C} bins x {T} tasks")
    partial = torch.empty(max(pdoubles, 1), dtype=torch.float64, device=dev)
    Gs = torch.zeros(T * NN, dtype=torch.float64, device=dev)
    Hs = torch.zeros_like(Gs)
    mpart = torch.zeros(5 * 4096, dtype=torch.float64, device=dev)  # train + up to 4 eval sets (fused launch)
    status = torch.zeros(R * T * NN, dtype=torch.int8, device=dev)
    feat = torch.zeros(R * T * NN, dtype=torch.int16, device=dev)
    sbin = torch.zeros(R * T * NN, dtype=torch.uint8, device=dev)
    leaf = torch.zeros(R * T * NN, dtype=torch.float32, device=dev)
    gain = torch.zeros_like(leaf)
    cover = torch.zeros_like(leaf)
    hist = torch.zeros(R * (1 + len(ev_names)), dtype=torch.float32, device=dev)
    history = []
    if dp is not None:
        _fit_dp_rounds(model, dp, d_bins, d_Y, n, F, cells, T, margin, ev_names, ev_keep, g, h, node, partial, Gs, Hs,
                       mpart, status, feat, sbin, leaf, gain, cover, history, stream)
    r0 = R if dp is not None else 0
    qbits = quant_bits(model.objective, n, model.hist_mode, dp is not None)
    model.quant_bits_used = qbits
    while r0 < R:
        r1 = min(R, r0 + rounds_per_call)
        N.call("em_gbdt_fit", d_bins.data_ptr(), d_Y.data_ptr(), n, F, cells.hp, cells.dev.data_ptr(), T,
               margin.data_ptr(), ev_structs,
               len(ev_names), r0, r1, D, OBJ[model.objective], MET[model.eval_metric], model.eta, model.lam,
               model.gamma, model.mcw, model.subsample, model.seed & 0xFFFFFFFF, g.data_ptr(), h.data_ptr(),
               node.data_ptr(), node2.data_ptr(), partial.data_ptr(), partial.numel(), Gs.data_ptr(), Hs.data_ptr(), mpart.data_ptr(),
               status.data_ptr(), feat.data_ptr(), sbin.data_ptr(), leaf.data_ptr(), gain.data_ptr(),
               cover.data_ptr(), hist.data_ptr(), qbits,
               # separate launches instead of the fused round (bit-identity tests; csrc/gbdt.hip), and the
               # opt-in fused levels (splits inside the next level's histogram pass, EM_GBDT_PRESPLIT)
               (1 if getattr(model, "separate_launches", False) else 0)
               | (2 if getattr(model, "presplit_levels", False) else 0), stream)
        hh = hist.view(R, 1 + len(ev_names))[r0:r1].cpu().numpy()
        for i, rnd in enumerate(range(r0, r1)):
            rec = {"round": rnd}
            # XGBoost4J watch order: evals only (train appears if the caller passed it as a watch)
            for j, name in enumerate(ev_names):
                rec[name] = float(hh[i, 1 + j])
            history.append(rec)
            model._log_round(rec)
        r0 = r1
    # the host copy of the ensemble: dtypes converted on the device, one packed device-to-host copy,
    # numpy views of it (per-array host conversions of ~0.5 M nodes cost several ms)
    # (widest dtypes first: every view starts aligned)
    parts = [leaf.to(torch.float64), gain.to(torch.float64), cover.to(torch.float64), feat.to(torch.int32),
             sbin.to(torch.int32), status]
    host = torch.cat([t.reshape(-1).view(torch.uint8) for t in parts]).cpu().numpy()
    arrs, o = [], 0
    for t, dt in zip(parts, (np.float64, np.float64, np.float64, np.int32, np.int32, np.int8)):
        nb = t.numel() * t.element_size()
        arrs.append(host[o:o + nb].view(dt).reshape(R * T, NN))
        o += nb
    lf, gn, cv, fe, sb, st = arrs
    # a histogram block that waited past its bound for its task's splits (the fused levels of em_gbdt_fit,
    # csrc/gbdt.hip HistPre) leaves invalid trees: fail loudly instead of returning them
    if N.query("em_gbdt_fused_error") != 0:
        raise RuntimeError("GPU GBDT: a fused level's wait for its task's splits timed out (trees invalid)")
    trees = TreeArrays.from_arrays(D, st, fe, sb, lf, gn, cv)
    model._device_trees = (status, feat, sbin, leaf)
    return trees, history


def _fit_dp_rounds(model, dp, d_bins, d_Y, n, F, cells, T, margin, ev_names, ev_keep, g, h, node, partial, Gs, Hs,
                   mpart, status, feat, sbin, leaf, gain, cover, history, stream):
    """C4: per-level histogram all-reduce between the HIP hist and split kernels (stream-ordered,
    no host sync inside a round); metric sums are all-reduced and read back once at the end."""
    import torch.distributed as dist

    R, D = model.nround, model.max_depth
    NN = 2 ** (D + 1) - 1
    dev = d_bins.device
    seed = (model.seed + 0x9E3779B9 * dp.rank) & 0xFFFFFFFF
    msum = torch.zeros(R, max(1, len(ev_names)), 2, dtype=torch.float64, device=dev)
    S = ctypes.c_int64(0)
    obj, met = OBJ[model.objective], MET[model.eval_metric]

    def off(t, k):  # pointer to round-k slice of a [R*T*NN] buffer
        return t.data_ptr() + k * T * NN * t.element_size()

    for rnd in range(R):
        N.call("em_gbdt_dp_round_begin", rnd, T, n, D, margin.data_ptr(), d_Y.data_ptr(), g.data_ptr(), h.data_ptr(),
               node.data_ptr(), obj, model.subsample, seed, off(status, rnd), off(feat, rnd), off(sbin, rnd),
               off(gain, rnd), stream)
        for level in range(D):
            N.call("em_gbdt_dp_level_hist", level, d_bins.data_ptr(), g.data_ptr(), h.data_ptr(), node.data_ptr(), T, n,
                   F, cells.hp, cells.dev.data_ptr(), partial.data_ptr(), partial.numel(), ctypes.byref(S), stream)
            dist.all_reduce(partial[:S.value], group=dp.group)
            N.call("em_gbdt_dp_level_split", level, d_bins.data_ptr(), partial.data_ptr(), T, n, F,
                   cells.dev.data_ptr(), cells.C, D,
                   node.data_ptr(), Gs.data_ptr(), Hs.data_ptr(), off(status, rnd), off(feat, rnd), off(sbin, rnd),
                   off(gain, rnd), model.lam, model.mcw, stream)
        N.call("em_gbdt_dp_round_end", T, n, D, margin.data_ptr(), node.data_ptr(), off(status, rnd), off(feat, rnd),
               off(gain, rnd), Gs.data_ptr(), Hs.data_ptr(), off(leaf, rnd), off(cover, rnd), model.lam, model.gamma,
               model.eta, stream)
        for j, name in enumerate(ev_names):
            db, dy, em = ev_keep[3 * j:3 * j + 3]
            ne = db.shape[0]
            N.call("em_gbdt_predict", db.data_ptr(), em.data_ptr(), T, ne, F, D, rnd * T, rnd * T + T,
                   status.data_ptr(), feat.data_ptr(), sbin.data_ptr(), leaf.data_ptr(), stream)
            N.call("em_gbdt_metric_sum", em.data_ptr(), dy.data_ptr(), T, ne, obj, met, mpart.data_ptr(),
                   msum[rnd, j, :1].data_ptr(), stream)
            msum[rnd, j, 1] = float(ne if met >= 3 else T * ne)
    if ev_names:
        dist.all_reduce(msum, group=dp.group)
    ms = msum.cpu().numpy()
    for rnd in range(R):
        rec = {"round": rnd}
        for j, name in enumerate(ev_names):
            v = ms[rnd, j, 0] / max(ms[rnd, j, 1], 1.0)
            rec[name] = float(np.sqrt(v)) if model.eval_metric == "rmse" else float(v)
        history.append(rec)
        model._log_round(rec)


def predict_margin(model, X):
    dev = _dev()
    tr = model.trees
    bins = apply_bins(X, model.cuts)
    n, F = bins.shape
    T = model.n_tasks
    NN = 2 ** (tr.max_depth + 1) - 1
    dt = getattr(model, "_device_trees", None)
    if dt is None:
        dt = (torch.from_numpy(tr.status.reshape(-1)).to(dev), torch.from_numpy(tr.feat.astype(np.int16).reshape(-1)).to(dev),
              torch.from_numpy(tr.sbin.astype(np.uint8).reshape(-1)).to(dev),
              torch.from_numpy(tr.leaf.astype(np.float32).reshape(-1)).to(dev))
        model._device_trees = dt
    status, feat, sbin, leaf = dt
    d_bins = torch.from_numpy(np.ascontiguousarray(bins, dtype=np.uint8)).to(dev)
    margin = torch.full((T * n,), float(model.base_margin), dtype=torch.float32, device=dev)
    N.call("em_gbdt_predict", d_bins.data_ptr(), margin.data_ptr(), T, n, F, tr.max_depth, 0, tr.n_trees,
           status.data_ptr(), feat.data_ptr(), sbin.data_ptr(), leaf.data_ptr(), N.stream_handle(dev))
    return margin.view(T, n).t().cpu().numpy().astype(np.float64)
