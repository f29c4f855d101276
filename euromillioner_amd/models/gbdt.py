"""Gradient-boosted trees with XGBoost ``gbtree`` semantics (the reference's learner).

Reference: ``Main.java:113-141`` trains ``XGBoost.train(..., nround=500)`` with
``booster=gbtree, eta=1.0, max_depth=3, objective=reg:logistic, subsample=1,
gamma=1.0, eval_metric=logloss`` (``lambda=1``, ``min_child_weight=1``,
``base_score=0.5`` are XGBoost defaults) and predicts with ``cpu_predictor``.
Upstream XGBoost runs this in C++ (libxgboost via JNI); here:

* ``backend="hip"`` — a device-resident engine (``csrc/gbdt.hip``): per round a
  gradient kernel, per level a deterministic histogram kernel (K8), a split-scan
  kernel (K9), a partition kernel (K10), then prune/leaf/margin-update (K12) and a
  fused metric reduction (K13); prediction is the tree-ensemble kernel (K11).  The
  C++ driver runs all rounds without host round-trips.
* ``backend="numpy"`` — the oracle used by the tests and on CPU-only machines.

Split finding is histogram-based over per-feature cut points.  When a feature has
at most ``max_bin`` distinct values (true for every reference feature: dow 7,
month 12, day 31, year 17, numbers <= 50, stars <= 12) the cut points are the
midpoints between consecutive distinct values, so the candidate splits — and hence
the trees — are exactly those of XGBoost's exact-greedy updater
(``tests/test_gbdt.py::test_hist_equals_exact``).

Semantics implemented (XGBoost 1.x ``ColMaker`` + ``TreePruner``):
* loss_chg = G_L^2/(H_L+l) + G_R^2/(H_R+l) - G^2/(H+l); a node splits only if
  loss_chg > 1e-6 and both children have hessian sum >= min_child_weight;
  ties keep the lower feature index (then the lower cut);
* bottom-up pruning: a split whose children are both leaves is removed while
  loss_chg < gamma (``min_split_loss``);
* leaf value = -G/(H+l) * eta; margins start at logit(base_score);
* reg:logistic/binary:logistic: g = p - y, h = max(p(1-p), 1e-16), labels must be
  in [0, 1] (XGBoost raises otherwise); reg:squarederror: g = m - y, h = 1.

Multiple targets (``Y [n, T]``) train T independent boosters in lock-step (the
default "next-draw" task: one booster per number/star, 62 in all).
"""
from __future__ import annotations

import json
import math

import numpy as np

KRT_EPS = 1e-6
OBJECTIVES = ("reg:logistic", "binary:logistic", "reg:squarederror", "multi:softprob", "multi:softmax")
MULTI = ("multi:softprob", "multi:softmax")


# ----------------------------------------------------------------------------- binning
def make_cuts(X: np.ndarray, max_bin: int = 256) -> list[np.ndarray]:
    """Per-feature split values.  bin(x) = number of cuts < x ... i.e. searchsorted(cuts, x, 'left')
    with rows going LEFT of cut c when x < cuts[c]."""
    cuts = []
    for f in range(X.shape[1]):
        col = X[:, f]
        col = col[~np.isnan(col)]
        u = np.unique(col)
        if len(u) <= 1:
            cuts.append(np.zeros(0, dtype=np.float64))
            continue
        if len(u) <= max_bin:
            c = (u[:-1].astype(np.float64) + u[1:].astype(np.float64)) * 0.5
        else:
            qs = np.quantile(col.astype(np.float64), np.linspace(0, 1, max_bin + 1)[1:-1])
            c = np.unique(qs)
        cuts.append(c)
    return cuts


class _DP:
    """C4 helper: histogram / sum all-reduce for data-parallel boosting (every rank holds a row
    shard; identical global sums give identical splits, so trees need no broadcast)."""

    def __init__(self, group):
        import torch.distributed as dist

        self.dist, self.group = dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.nccl = dist.get_backend(group) == "nccl"

    def sum_(self, arr: np.ndarray) -> np.ndarray:
        import torch

        t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float64))
        if self.nccl:
            t = t.cuda()
        self.dist.all_reduce(t, group=self.group)
        return t.cpu().numpy().reshape(np.shape(arr))

    def gather(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out


def make_cuts_dp(X: np.ndarray, max_bin: int, dp: "_DP") -> list[np.ndarray]:
    """Global cuts from per-rank value summaries.  Exact (== single-process cuts) whenever a
    feature has <= 16*max_bin distinct values per rank and <= max_bin globally (true for draw
    data); otherwise a merged quantile summary."""
    summaries = []
    for f in range(X.shape[1]):
        col = X[:, f]
        u = np.unique(col[~np.isnan(col)])
        if len(u) > 16 * max_bin:
            u = np.unique(np.quantile(u, np.linspace(0, 1, 16 * max_bin)))
        summaries.append(u)
    merged = dp.gather(summaries)
    cols = [np.unique(np.concatenate([m[f] for m in merged])) for f in range(X.shape[1])]
    width = max((len(c) for c in cols), default=0)
    Xm = np.full((max(width, 1), X.shape[1]), np.nan)
    for f, c in enumerate(cols):
        Xm[:len(c), f] = c
    return make_cuts(Xm, max_bin)


def apply_bins(X: np.ndarray, cuts: list[np.ndarray]) -> np.ndarray:
    """bin index per value: number of cuts strictly below x (x < cut -> left of it)."""
    n, F = X.shape
    nb = max((len(c) for c in cuts), default=0) + 1
    dtype = np.uint8 if nb <= 256 else np.uint16
    out = np.zeros((n, F), dtype=dtype)
    for f in range(F):
        if len(cuts[f]):
            out[:, f] = np.searchsorted(cuts[f], X[:, f], side="right")
    return out


# ----------------------------------------------------------------------------- trees
class TreeArrays:
    """Heap-numbered trees: node i has children 2i+1 / 2i+2.  status 0 unused, 1 split, 2 leaf."""

    def __init__(self, n_trees: int, max_depth: int):
        nn = 2 ** (max_depth + 1) - 1
        self.max_depth = max_depth
        self.feat = np.full((n_trees, nn), -1, dtype=np.int32)
        self.sbin = np.zeros((n_trees, nn), dtype=np.int32)  # go left iff bin <= sbin
        self.split_value = np.zeros((n_trees, nn), dtype=np.float64)  # go left iff x < split_value
        self.status = np.zeros((n_trees, nn), dtype=np.int8)
        self.leaf = np.zeros((n_trees, nn), dtype=np.float64)
        self.gain = np.zeros((n_trees, nn), dtype=np.float64)
        self.cover = np.zeros((n_trees, nn), dtype=np.float64)

    @classmethod
    def from_arrays(cls, max_depth: int, status, feat, sbin, leaf, gain, cover) -> "TreeArrays":
        """Wrap existing [n_trees, nn] arrays (int8 / int32 / int32 / float64 x 3) without copying."""
        t = cls.__new__(cls)
        t.max_depth = max_depth
        t.status, t.feat, t.sbin, t.leaf, t.gain, t.cover = status, feat, sbin, leaf, gain, cover
        t.split_value = np.zeros(feat.shape, dtype=np.float64)
        return t

    @property
    def n_trees(self):
        return self.feat.shape[0]

    def set_split_values(self, cuts):
        """split_value = cuts[feat][sbin] at every split node (one gather over a flattened cut table)."""
        t, i = np.nonzero(self.status == 1)
        if t.size == 0:
            return
        off = np.concatenate([[0], np.cumsum([len(c) for c in cuts])]).astype(np.int64)
        flat = np.concatenate([np.asarray(c, np.float64) for c in cuts] + [np.zeros(1)])
        self.split_value[t, i] = flat[off[self.feat[t, i]] + self.sbin[t, i]]


def predict_margin_values(trees: TreeArrays, X: np.ndarray, tree_task: np.ndarray, n_tasks: int,
                          base_margin: float) -> np.ndarray:
    """Raw-value traversal (cpu_predictor equivalent): margin[n, T]."""
    n = X.shape[0]
    out = np.full((n, n_tasks), base_margin, dtype=np.float64)
    rows = np.arange(n)
    for k in range(trees.n_trees):
        node = np.zeros(n, dtype=np.int64)
        for _ in range(trees.max_depth + 1):
            st = trees.status[k, node]
            sp = st == 1
            if not sp.any():
                break
            f = trees.feat[k, node[sp]]
            go_right = ~(X[rows[sp], f] < trees.split_value[k, node[sp]])
            node[sp] = 2 * node[sp] + 1 + go_right
        out[:, tree_task[k]] += trees.leaf[k, node]
    return out


# ----------------------------------------------------------------------------- objectives
def _sigmoid(x):
    """1 / (1 + exp(-x)) in x's dtype, exactly the HIP kernels' form (csrc/gbdt.hip:99, :1255) so trees stay
    bit-identical.  For margins below the dtype's exp range exp(-x) is +inf and the result the correct
    0.0: that overflow is expected here, so it is silenced for this expression only."""
    with np.errstate(over="ignore"):
        return 1.0 / (1.0 + np.exp(-x))


def base_margin_for(objective: str, base_score: float) -> float:
    if objective in ("reg:logistic", "binary:logistic"):
        return float(math.log(base_score / (1.0 - base_score)))
    return float(base_score)


def softmax_rows(margin: np.ndarray) -> np.ndarray:
    """Row softmax over the class margins in float32, classes summed in order (== the HIP kernel)."""
    m = np.asarray(margin, dtype=np.float32)
    mx = m[:, :1].copy()
    for k in range(1, m.shape[1]):
        mx = np.maximum(mx, m[:, k:k + 1])
    e = np.exp(m - mx)
    s = np.zeros_like(mx)
    for k in range(m.shape[1]):
        s += e[:, k:k + 1]
    return e / s


def transform(objective: str, margin: np.ndarray) -> np.ndarray:
    if objective in ("reg:logistic", "binary:logistic"):
        return _sigmoid(margin)
    if objective in MULTI:
        return softmax_rows(margin)
    return margin


def check_labels(objective: str, y: np.ndarray, num_class: int = 0) -> None:
    if objective in MULTI:
        yy = np.asarray(y).reshape(-1)
        if np.any(np.isnan(yy)) or np.any(yy < 0) or np.any(yy != np.floor(yy)) or \
                (num_class and np.any(yy >= num_class)):
            # XGBoost: SoftmaxMultiClassObj -> "label must be in [0, num_class)"
            raise ValueError("multi-class labels must be integers in [0, num_class)")
        return
    if objective in ("reg:logistic", "binary:logistic"):
        if np.any((y < 0) | (y > 1)) or np.any(np.isnan(y)):
            # XGBoost: LogisticRegression::CheckLabel -> XGBoostError
            raise ValueError("label must be in [0,1] for logistic regression")


def gradients(objective: str, margin: np.ndarray, y: np.ndarray):
    if objective in ("reg:logistic", "binary:logistic"):
        p = _sigmoid(margin)
        return p - y, np.maximum(p * (p.dtype.type(1) - p), p.dtype.type(1e-16))
    if objective == "reg:squarederror":
        return margin - y, np.ones_like(margin)
    if objective in MULTI:  # y one-hot [n, K]
        p = softmax_rows(margin)
        return p - y, np.maximum(np.float32(2) * p * (np.float32(1) - p), np.float32(1e-16))
    raise ValueError(f"unsupported objective {objective}")


# ----------------------------------------------------------------------------- histogram modes
HIST_MODES = ("auto", "exact", "quant")
QUANT_MIN_ROWS = 32768  # "auto": fixed-point histograms from this many rows on (reference config: 928 rows -> exact)
_QUANT_SPLIT = 26  # oracle: q = hi * 2^26 + lo, so both halves' float64 GEMM sums stay exact integers


def quant_bits(objective: str, n: int, mode: str = "auto", distributed: bool = False) -> int:
    """Fixed-point scale s of the histogram sums (0 = exact fp64 sums).

    Quantised form (csrc/gbdt.hip gbdt_hist_q): q = rint(x * 2^s) per row for x in {g, h}; the
    logistic and softmax objectives have |g| <= 1 and 0 < h <= 0.5, so with n < 2^(61-s) every sum
    of q over rows stays below 2^61 and integer accumulation is exact in any order.  s = 61 -
    ceil(log2(n+1)) keeps 2^-s at or below the float32 ulp of any |g| >= 2^-20.  Squared error
    (unbounded g) and the data-parallel path (fp64 all-reduce of the histograms) stay exact."""
    if mode not in HIST_MODES:
        raise ValueError(f"hist_mode must be one of {HIST_MODES}")
    if mode == "exact" or distributed or objective == "reg:squarederror":
        return 0
    if (mode == "auto" and n < QUANT_MIN_ROWS) or n >= 1 << 26:
        return 0
    return 61 - max(1, int(n).bit_length())  # bit_length(n) == ceil(log2(n + 1))


def _quantise(x: np.ndarray, s: int) -> np.ndarray:
    return np.rint(x.astype(np.float64) * (2.0 ** s)).astype(np.int64)


def _quantise_h(h: np.ndarray, s: int) -> np.ndarray:
    """Hessians: a positive h never rounds to 0 (== csrc/gbdt.hip quantise_h).  The 1e-16 floor of a
    saturated row would, and a node of such rows would get H = 0 where the exact form keeps H > 0."""
    q = _quantise(h, s)
    return np.where((h > 0) & (q < 1), 1, q)


def _segment_cumsum(hist: np.ndarray, off: np.ndarray) -> np.ndarray:
    """Left sums "bins <= b" within each feature's cell segment [off[f], off[f+1]).  Per segment, so
    an int64 intermediate never exceeds one node's total (a cumsum over every feature's cells reaches
    F x the node total and would wrap past 2^63 near quant_bits' bound)."""
    out = np.empty_like(hist)
    for f in range(len(off) - 1):
        np.cumsum(hist[off[f]:off[f + 1]], axis=0, out=out[off[f]:off[f + 1]])
    return out


def _int_hist(onehot: np.ndarray, Zq: np.ndarray) -> np.ndarray:
    """Exact onehot.T @ Zq for int64 Zq (|entries| <= 2^s, n rows, quant_bits' bound n * 2^s < 2^61,
    n < 2^26): two float64 GEMMs of the 26-bit halves, whose partial sums are integers below 2^53 in
    any order."""
    hi = Zq >> _QUANT_SPLIT
    lo = Zq & ((1 << _QUANT_SPLIT) - 1)
    return ((onehot.T @ hi.astype(np.float64)).astype(np.int64) << _QUANT_SPLIT) + \
        (onehot.T @ lo.astype(np.float64)).astype(np.int64)


# ----------------------------------------------------------------------------- numpy oracle
def _best_split_hist(hg, hh, G, H, lam, mcw):
    """hg/hh: [F, B] node histograms.  Returns (gain, f, bin, GL, HL) or None."""
    cg = np.cumsum(hg, axis=1)[:, :-1]  # left = bins <= b
    ch = np.cumsum(hh, axis=1)[:, :-1]
    if cg.size == 0:
        return None
    gr, hr = G - cg, H - ch
    ok = (ch >= mcw) & (hr >= mcw)
    root = G * G / (H + lam)
    gain = np.where(ok, cg * cg / (ch + lam) + gr * gr / (hr + lam) - root, -np.inf)
    # first max in (feature, bin) order == lower feature index wins ties
    flat = int(np.argmax(gain))
    f, b = divmod(flat, gain.shape[1])
    g = float(gain[f, b])
    if not np.isfinite(g) or g <= KRT_EPS:
        return None
    return g, f, b, float(cg[f, b]), float(ch[f, b])


def grow_tree_numpy(bins, nbins, g, h, max_depth, lam, mcw, gamma, eta, trees: TreeArrays, k: int):
    n, F = bins.shape
    node = np.zeros(n, dtype=np.int64)
    G = np.zeros(2 ** (max_depth + 1) - 1)
    H = np.zeros_like(G)
    G[0], H[0] = g.astype(np.float64).sum(), h.astype(np.float64).sum()
    trees.status[k, 0] = 2
    for depth in range(max_depth):
        for i in range(2 ** depth - 1, 2 ** (depth + 1) - 1):
            if trees.status[k, i] != 2:
                continue
            sel = node == i
            if not sel.any():
                continue
            hg = np.zeros((F, nbins))
            hh = np.zeros((F, nbins))
            bs = bins[sel]
            gs, hs = g[sel].astype(np.float64), h[sel].astype(np.float64)
            for f in range(F):
                hg[f] = np.bincount(bs[:, f], weights=gs, minlength=nbins)
                hh[f] = np.bincount(bs[:, f], weights=hs, minlength=nbins)
            best = _best_split_hist(hg, hh, G[i], H[i], lam, mcw)
            if best is None:
                continue
            gain, f, b, GL, HL = best
            trees.status[k, i] = 1
            trees.feat[k, i], trees.sbin[k, i], trees.gain[k, i] = f, b, gain
            l, r = 2 * i + 1, 2 * i + 2
            G[l], H[l], G[r], H[r] = GL, HL, G[i] - GL, H[i] - HL
            trees.status[k, l] = trees.status[k, r] = 2
            right = sel & (bins[:, f] > b)
            node[sel] = l
            node[right] = r
    _prune_and_leaves(trees, k, G, H, lam, gamma, eta, max_depth)
    trees.cover[k] = H
    return node


def _prune_and_leaves(trees: TreeArrays, k, G, H, lam, gamma, eta, max_depth):
    for i in range(2 ** max_depth - 2, -1, -1):  # bottom-up over internal slots
        if trees.status[k, i] == 1:
            l, r = 2 * i + 1, 2 * i + 2
            if trees.status[k, l] == 2 and trees.status[k, r] == 2 and trees.gain[k, i] < gamma:
                trees.status[k, i] = 2
                trees.status[k, l] = trees.status[k, r] = 0
                trees.feat[k, i] = -1
    for i in range(len(G)):
        if trees.status[k, i] == 2:
            trees.leaf[k, i] = np.float32(-G[i] / (H[i] + lam) * eta)  # leaf values are float (XGBoost)


def _leaf_of(trees: TreeArrays, k, node):
    node = node.copy()
    for _ in range(trees.max_depth + 1):
        bad = trees.status[k, node] != 2
        if not bad.any():
            break
        node[bad] = (node[bad] - 1) // 2
    return node


class GBDT:
    """XGBoost-semantics booster(s).  Y may be [n] or [n, T] (T boosters in lock-step)."""

    def __init__(self, eta=1.0, max_depth=3, objective="reg:logistic", subsample=1.0, gamma=1.0,
                 reg_lambda=1.0, min_child_weight=1.0, base_score=0.5, nround=500, max_bin=256,
                 eval_metric="logloss", seed=0, backend="auto", log=None, log_every=1, num_class=0, nthread=0,
                 hist_mode="auto"):
        if objective not in OBJECTIVES:
            raise ValueError(f"objective must be one of {OBJECTIVES}")
        self.eta, self.max_depth, self.objective = float(eta), int(max_depth), objective
        self.subsample, self.gamma, self.lam = float(subsample), float(gamma), float(reg_lambda)
        self.mcw, self.base_score, self.nround = float(min_child_weight), float(base_score), int(nround)
        self.max_bin, self.eval_metric, self.seed = int(max_bin), eval_metric, int(seed)
        self.num_class = int(num_class)
        self.nthread = int(nthread)  # XGBoost nthread (Main.java:122): CPU threads of the numpy engine (0 = all)
        if objective in MULTI and eval_metric in ("logloss", "error"):
            self.eval_metric = "m" + eval_metric  # XGBoost's multi-class defaults: mlogloss / merror
        self.backend = backend
        if hist_mode not in HIST_MODES:
            raise ValueError(f"hist_mode must be one of {HIST_MODES}")
        self.hist_mode = hist_mode  # histogram sums: exact fp64 or fixed point (quant_bits); both engines agree
        self.log, self.log_every = log, log_every
        self.trees: TreeArrays | None = None
        self.cuts = None
        self.num_feature = None
        self.n_tasks = 1
        self.history: list[dict] = []

    @classmethod
    def from_params(cls, params: dict, nround: int = 500, **kw):
        """Build from the reference's parameter map (Main.java:113-126)."""
        p = dict(params)
        if p.get("booster", "gbtree") != "gbtree":
            raise ValueError("only booster=gbtree is supported")
        args = dict(eta=float(p.get("eta", 0.3)), max_depth=int(p.get("max_depth", 6)),
                    objective=p.get("objective", "reg:squarederror"), subsample=float(p.get("subsample", 1)),
                    gamma=float(p.get("gamma", 0.0)), reg_lambda=float(p.get("lambda", 1.0)),
                    min_child_weight=float(p.get("min_child_weight", 1.0)),
                    base_score=float(p.get("base_score", 0.5)), eval_metric=p.get("eval_metric", "logloss"),
                    nround=nround, num_class=int(p.get("num_class", 0)), nthread=int(p.get("nthread", 0)))
        args.update(kw)
        return cls(**args)

    @property
    def base_margin(self) -> float:
        return base_margin_for(self.objective, self.base_score)

    def _resolve_backend(self):
        if self.backend != "auto":
            return self.backend
        try:
            import torch

            if torch.cuda.is_available():
                from ..ops import _native

                _native.lib()
                return "hip"
        except Exception:  # noqa: BLE001
            pass
        return "numpy"

    def fit(self, X: np.ndarray, Y: np.ndarray, evals: dict | None = None, group=None):
        """``group``: a torch.distributed process group -> data-parallel boosting (C4): X/Y and every
        eval set are this rank's row shard; histograms, node sums and metrics are all-reduced."""
        X = np.asarray(X, dtype=np.float64)
        Y = np.asarray(Y, dtype=np.float64)
        dp = _DP(group) if group is not None else None
        if self.objective in MULTI:  # class ids -> one booster per class on one-hot targets
            y = Y.reshape(-1)
            ev_y = {k: np.asarray(ey, np.float64).reshape(-1) for k, (_, ey) in (evals or {}).items()}
            for v in (y, *ev_y.values()):
                check_labels(self.objective, v, self.num_class)
            if not self.num_class:  # XGBoost requires num_class; 0 = infer (global max under DP)
                top = max([float(v.max()) for v in (y, *ev_y.values()) if v.size] or [0.0])
                if dp is not None:
                    top = float(dp.sum_(np.eye(dp.world)[dp.rank] * top).max())  # all-gather of per-rank maxima
                self.num_class = int(top) + 1
            eye = np.eye(self.num_class, dtype=np.float64)
            Y = eye[y.astype(np.int64)]
            evals = {k: (ex, eye[ev_y[k].astype(np.int64)]) for k, (ex, _) in (evals or {}).items()}
        if Y.ndim == 1:
            Y = Y[:, None]
        check_labels(self.objective, Y)
        self.n_tasks = Y.shape[1]
        self.cuts = make_cuts_dp(X, self.max_bin, dp) if dp is not None else make_cuts(X, self.max_bin)
        bins = apply_bins(X, self.cuts)
        nbins = max((len(c) for c in self.cuts), default=0) + 1
        evals = evals or {}
        backend = self._resolve_backend()
        self.backend_used = backend
        if backend == "hip":
            from . import gbdt_hip

            try:
                self.trees, self.history = gbdt_hip.fit(self, X, bins, nbins, Y, evals, dp=dp)
            except gbdt_hip.PlanUnsupported as e:
                if self.backend != "auto":
                    raise
                from .. import log as L

                L.get("GBDT").warning("%s; training on the numpy engine", e)
                backend = self.backend_used = "numpy"
        if backend != "hip":
            from threadpoolctl import threadpool_limits

            with threadpool_limits(limits=self.nthread or None):  # X3: the reference's OpenMP nthread
                self.trees, self.history = self._fit_numpy(X, bins, nbins, Y, evals, dp=dp)
        self.trees.set_split_values(self.cuts)
        return self

    def _fit_numpy(self, X, bins, nbins, Y, evals, dp=None):
        """Oracle, vectorised over tasks and nodes: per level one GEMM of the one-hot bin matrix
        [n, sum(bins)] with (g, h) scattered by (task, node)."""
        n, T = Y.shape
        R, D = self.nround, self.max_depth
        NN = 2 ** (D + 1) - 1
        F = bins.shape[1]
        trees = TreeArrays(R * T, D)
        # float32 margins / gradients, float64 histogram sums: XGBoost's GradientPair / GradStats
        margin = np.full((n, T), self.base_margin, dtype=np.float32)
        ev_margin = {k: np.full((len(v[0]), T), self.base_margin, dtype=np.float32) for k, v in evals.items()}
        ev_bins = {k: apply_bins(np.asarray(v[0], np.float64), self.cuts) for k, v in evals.items()}
        Y32 = Y.astype(np.float32)
        nbf = np.array([len(c) + 1 for c in self.cuts])
        off = np.concatenate([[0], np.cumsum(nbf)])
        onehot = np.zeros((n, off[-1]), dtype=np.float64)
        for f in range(F):
            onehot[np.arange(n), off[f] + bins[:, f]] = 1.0
        row_feat = np.repeat(np.arange(F), nbf)
        rowseg_start = off[row_feat]
        valid_row = (np.arange(off[-1]) - rowseg_start) < (nbf[row_feat] - 1)  # not the last bin of a feature
        rng = np.random.default_rng(self.seed if dp is None else [self.seed, dp.rank])
        red = dp.sum_ if dp is not None else (lambda a: a)
        hist = []
        tix = np.arange(T)
        qs = quant_bits(self.objective, n, self.hist_mode, dp is not None)
        inv = 2.0 ** -qs
        self.quant_bits_used = qs
        for rnd in range(R):
            g, h = gradients(self.objective, margin, Y32)
            if self.subsample < 1.0:
                keep = (rng.random((n, T)) < self.subsample).astype(np.float32)
                g, h = g * keep, h * keep
            if qs:  # fixed point: integer sums, exact in any order (== gbdt_hist_q)
                g64, h64 = _quantise(g, qs), _quantise_h(h, qs)
            else:
                g64, h64 = g.astype(np.float64), h.astype(np.float64)
            node = np.zeros((n, T), dtype=np.int64)
            st = np.zeros((T, NN), np.int8)
            st[:, 0] = 2
            feat = np.full((T, NN), -1, np.int32)
            sbin = np.zeros((T, NN), np.int32)
            gain = np.zeros((T, NN))
            Gs = np.zeros((T, NN))
            Hs = np.zeros((T, NN))
            if not qs:
                Gs[:, 0], Hs[:, 0] = red(g64.sum(0)), red(h64.sum(0))
            for depth in range(D):
                first, nl = 2 ** depth - 1, 2 ** depth
                rel = node - first  # [n, T]
                act = (rel >= 0) & (rel < nl)
                col = np.where(act, tix[None, :] * nl + rel, 0)
                Zg = np.zeros((n, T * nl), dtype=g64.dtype)
                Zh = np.zeros((n, T * nl), dtype=h64.dtype)
                rows = np.nonzero(act)
                Zg[rows[0], col[rows]] = g64[rows]
                Zh[rows[0], col[rows]] = h64[rows]
                if qs:
                    HG, HH = _int_hist(onehot, Zg), _int_hist(onehot, Zh)
                else:
                    HG = red(onehot.T @ Zg)  # [sum bins, T*nl]; C4: all-reduced under DP
                    HH = red(onehot.T @ Zh)
                # segmented prefix sums: left sums for "bin <= b" of feature f, all columns at once
                if qs:  # integers: per feature segment (no intermediate beyond one node's total)
                    GL, HL = _segment_cumsum(HG, off), _segment_cumsum(HH, off)
                else:
                    CG, CH = np.cumsum(HG, axis=0), np.cumsum(HH, axis=0)
                    baseg = np.where(rowseg_start[:, None] > 0, CG[np.maximum(rowseg_start - 1, 0)], 0)
                    baseh = np.where(rowseg_start[:, None] > 0, CH[np.maximum(rowseg_start - 1, 0)], 0)
                    GL, HL = CG - baseg, CH - baseh
                cols_t = np.repeat(tix, nl)
                cols_i = np.tile(np.arange(nl), T) + first
                if qs:  # node totals = feature 0's cells; every sum converted to double once
                    Gnq, Hnq = GL[off[1] - 1], HL[off[1] - 1]
                    GR, HR = (Gnq[None, :] - GL).astype(np.float64) * inv, (Hnq[None, :] - HL).astype(np.float64) * inv
                    GL, HL = GL.astype(np.float64) * inv, HL.astype(np.float64) * inv
                    Gn, Hn = Gnq.astype(np.float64) * inv, Hnq.astype(np.float64) * inv
                    if depth == 0:
                        Gs[:, 0], Hs[:, 0] = Gn, Hn
                else:
                    Gn, Hn = Gs[cols_t, cols_i], Hs[cols_t, cols_i]
                    GR, HR = Gn[None, :] - GL, Hn[None, :] - HL
                ok = valid_row[:, None] & (HL >= self.mcw) & (HR >= self.mcw) & (st[cols_t, cols_i] == 2)[None, :]
                with np.errstate(divide="ignore", invalid="ignore"):
                    gn = GL * GL / (HL + self.lam) + GR * GR / (HR + self.lam) - (Gn * Gn / (Hn + self.lam))[None, :]
                gn = np.where(ok, gn, -np.inf)
                br = np.argmax(gn, axis=0)  # first max: lower feature, then lower bin
                bv = gn[br, np.arange(gn.shape[1])]
                for c in np.nonzero(np.isfinite(bv) & (bv > KRT_EPS))[0]:
                    t, i, rrow = cols_t[c], cols_i[c], br[c]
                    f = row_feat[rrow]
                    st[t, i], feat[t, i], sbin[t, i], gain[t, i] = 1, f, rrow - off[f], bv[c]
                    l, r = 2 * i + 1, 2 * i + 2
                    st[t, l] = st[t, r] = 2
                    Gs[t, l], Hs[t, l] = GL[rrow, c], HL[rrow, c]
                    Gs[t, r], Hs[t, r] = GR[rrow, c], HR[rrow, c]
                # partition
                nd = node
                k = (st[tix[None, :], nd] == 1) & act
                fsel = feat[tix[None, :], nd]
                bsel = bins[np.arange(n)[:, None], np.maximum(fsel, 0)]
                child = 2 * nd + 1 + (bsel > sbin[tix[None, :], nd])
                node = np.where(k, child, nd)
            for t in range(T):
                kk = rnd * T + t
                trees.status[kk], trees.feat[kk], trees.sbin[kk], trees.gain[kk] = st[t], feat[t], sbin[t], gain[t]
                _prune_and_leaves(trees, kk, Gs[t], Hs[t], self.lam, self.gamma, self.eta, D)
                trees.cover[kk] = np.where(trees.status[kk] > 0, Hs[t], 0.0)
                margin[:, t] += trees.leaf[kk, _leaf_of(trees, kk, node[:, t])].astype(np.float32)
                for name, eb in ev_bins.items():
                    ev_margin[name][:, t] += trees.leaf[kk, _route_bins(trees, kk, eb)].astype(np.float32)
            rec = {"round": rnd}
            for name, (ex, ey) in evals.items():
                rec[name] = self._metric(np.asarray(ey, np.float64).reshape(len(ex), -1), ev_margin[name], dp)
            hist.append(rec)
            self._log_round(rec)
        return trees, hist

    def _metric(self, y, margin, dp=None):
        from .. import metrics as M

        p = transform(self.objective, margin)
        if dp is None:
            return M.EVAL_METRICS[self.eval_metric](y, p)
        # global mean from per-rank (sum, count): rmse averages squares before the root
        y = np.asarray(y, np.float64).reshape(-1)
        p = np.asarray(p, np.float64).reshape(-1)
        if self.eval_metric in ("mlogloss", "merror"):
            yy = np.asarray(y, np.float64).reshape(-1, self.n_tasks)
            pp = np.asarray(p, np.float64).reshape(-1, self.n_tasks)
            loc = float(M.EVAL_METRICS[self.eval_metric](yy, pp) * len(yy)) if len(yy) else 0.0
            tot = dp.sum_(np.array([loc, float(len(yy))]))
            return float(tot[0] / max(tot[1], 1.0))
        if self.eval_metric == "rmse":
            loc = float(np.sum((y - p) ** 2))
        elif self.eval_metric == "error":
            loc = float(np.sum((p > 0.5).astype(np.float64) != y))
        else:
            loc = float(M.logloss(y, p) * y.size) if y.size else 0.0
        tot = dp.sum_(np.array([loc, float(y.size)]))
        m = tot[0] / max(tot[1], 1.0)
        return float(np.sqrt(m)) if self.eval_metric == "rmse" else float(m)

    def _log_round(self, rec):
        if self.log is None or (rec["round"] % self.log_every and rec["round"] != self.nround - 1):
            return
        parts = [f"[{rec['round']}]"] + [f"{k}-{self.eval_metric}:{v:.6f}" for k, v in rec.items() if k != "round"]
        self.log.info("\t".join(parts))

    # ------------------------------------------------------------------ inference
    def predict_margin(self, X: np.ndarray, backend: str | None = None) -> np.ndarray:
        X = np.asarray(X, dtype=np.float64)
        be = backend or getattr(self, "backend_used", "numpy")
        if be == "hip":
            from . import gbdt_hip

            return gbdt_hip.predict_margin(self, X)
        task = np.arange(self.trees.n_trees) % self.n_tasks
        return predict_margin_values(self.trees, X, task, self.n_tasks, self.base_margin)

    def predict(self, X: np.ndarray, backend: str | None = None) -> np.ndarray:
        """Like Booster.predict: float32 [n, T] (reg:logistic -> probabilities; multi:softprob ->
        class probabilities; multi:softmax -> the predicted class id, shape [n])."""
        p = transform(self.objective, self.predict_margin(X, backend)).astype(np.float32)
        if self.objective == "multi:softmax":
            return np.argmax(p, axis=1).astype(np.float32)
        return p

    # ------------------------------------------------------------------ persistence
    def to_json(self) -> dict:
        """XGBoost-JSON-like dump (learner/gradient_booster/model/trees)."""
        tr = self.trees
        trees = []
        for k in range(tr.n_trees):
            nodes = []
            for i in np.nonzero(tr.status[k])[0]:
                nd = {"nodeid": int(i), "cover": float(tr.cover[k, i])}
                if tr.status[k, i] == 1:
                    nd.update(split=f"f{int(tr.feat[k, i])}", split_condition=float(tr.split_value[k, i]),
                              yes=int(2 * i + 1), no=int(2 * i + 2), gain=float(tr.gain[k, i]))
                else:
                    nd["leaf"] = float(tr.leaf[k, i])
                nodes.append(nd)
            trees.append({"id": k, "task": int(k % self.n_tasks), "nodes": nodes})
        return {"learner": {"objective": self.objective, "base_score": self.base_score,
                            "num_target": self.n_tasks, "num_class": self.num_class,
                            "num_feature": len(self.cuts) if self.cuts is not None else self.num_feature,
                            "params": {"eta": self.eta, "max_depth": self.max_depth, "gamma": self.gamma,
                                       "lambda": self.lam, "min_child_weight": self.mcw,
                                       "subsample": self.subsample, "nround": self.nround},
                            "gradient_booster": {"name": "gbtree", "model": {"trees": trees}}}}

    def save(self, path: str) -> None:
        with open(path, "w", encoding="utf-8") as f:
            json.dump(self.to_json(), f)

    @classmethod
    def load(cls, path: str) -> "GBDT":
        with open(path, encoding="utf-8") as f:
            d = json.load(f)["learner"]
        p = d["params"]
        m = cls(eta=p["eta"], max_depth=p["max_depth"], objective=d["objective"], gamma=p["gamma"],
                reg_lambda=p["lambda"], min_child_weight=p["min_child_weight"], base_score=d["base_score"],
                nround=p["nround"], subsample=p.get("subsample", 1.0), backend="numpy")
        m.n_tasks = d["num_target"]
        m.num_class = int(d.get("num_class", 0))
        m.num_feature = d.get("num_feature")
        trees = d["gradient_booster"]["model"]["trees"]
        tr = TreeArrays(len(trees), m.max_depth)
        for k, t in enumerate(trees):
            for nd in t["nodes"]:
                i = nd["nodeid"]
                tr.cover[k, i] = nd.get("cover", 0.0)
                if "leaf" in nd:
                    tr.status[k, i], tr.leaf[k, i] = 2, nd["leaf"]
                else:
                    tr.status[k, i] = 1
                    tr.feat[k, i] = int(nd["split"][1:])
                    tr.split_value[k, i] = nd["split_condition"]
                    tr.gain[k, i] = nd.get("gain", 0.0)
        m.trees = tr
        m.backend_used = "numpy"
        return m


def _route_bins(trees: TreeArrays, k: int, bins: np.ndarray) -> np.ndarray:
    n = bins.shape[0]
    node = np.zeros(n, dtype=np.int64)
    rows = np.arange(n)
    for _ in range(trees.max_depth + 1):
        sp = trees.status[k, node] == 1
        if not sp.any():
            break
        f = trees.feat[k, node[sp]]
        node[sp] = 2 * node[sp] + 1 + (bins[rows[sp], f] > trees.sbin[k, node[sp]])
    return node


# ----------------------------------------------------------------------------- exact greedy (verification)
def exact_greedy_split(x: np.ndarray, g: np.ndarray, h: np.ndarray, lam: float, mcw: float):
    """XGBoost ColMaker enumeration on one feature: best (gain, threshold) over distinct values."""
    order = np.argsort(x, kind="stable")
    xs, gs, hs = x[order], g[order], h[order]
    G, H = gs.sum(), hs.sum()
    best = (-np.inf, None)
    GL = HL = 0.0
    for i in range(len(xs) - 1):
        GL += gs[i]
        HL += hs[i]
        if xs[i + 1] == xs[i]:
            continue
        GR, HR = G - GL, H - HL
        if HL < mcw or HR < mcw:
            continue
        gain = GL * GL / (HL + lam) + GR * GR / (HR + lam) - G * G / (H + lam)
        if gain > best[0]:
            best = (gain, (xs[i] + xs[i + 1]) * 0.5)
    return best
