"""Random forest over binary draw features (BASELINE config 4).

The reference declares Spark MLlib (``pom.xml:56-61``) and advertises "Random Forest"
(``README.md:6``) but never builds one.  This is a multi-output forest: inputs are the
62-wide multi-hot of the current draw (``lags`` draws -> 62*lags features), outputs
the 62-wide multi-hot of the next draw; each leaf stores the weighted mean 62-vector.

Semantics (shared bit-for-bit by the HIP engine ``csrc/forest.hip`` and the numpy
oracle below):

* Poisson(1) bootstrap weights per (tree, row) from a counter hash (Spark's scheme);
* per-node candidate features: ``k`` of ``F`` by a hashed partial Fisher-Yates
  (``feature_subset``: sqrt | log2 | all | onethird | <fraction>, Spark's rounding: ceil);
* split gain = weighted variance reduction summed over the 62 outputs (== Gini/2 per
  output): ``SL2/nL + SR2/nR - S2/n`` from exact integer sums; a split needs both
  children to weigh ``>= min_samples_leaf`` and a gain above rounding noise;
* complete-array trees: node ``i`` -> children ``2i+1`` (feature = 0), ``2i+2`` (= 1).

Tree-parallel data parallelism (C5): rank r builds the trees ``shard_range(T)`` with
global tree ids (so the forest is identical for any world size) and the packed arrays
are all-gathered.
"""
from __future__ import annotations

import json
import math

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
POISSON_CDF = (0.36787944117144233, 0.7357588823428847, 0.9196986029286058, 0.9810118431238463,
               0.9963401531726563, 0.9994058151824183, 0.999916758850712, 0.9999897508033253, 0.999998874797402)
CAND_SALT = 0x5EEDF00D


def mix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def hash3(seed, a, b):
    return mix64(mix64(np.uint64(seed) ^ mix64(a)) ^ np.asarray(b, dtype=np.uint64))


def poisson_weights(seed: int, tree: int, n: int) -> np.ndarray:
    h = hash3(seed, np.uint64((1 << 32) + tree), np.arange(n, dtype=np.uint64))
    u = (h >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    w = np.zeros(n, dtype=np.int64)
    for c in POISSON_CDF:
        w += (u >= c)
    return w


def candidates(seed: int, tree: int, node: int, F: int, k: int) -> np.ndarray:
    arr = list(range(F))
    key = np.uint64((tree << 32) | node)
    s = np.uint64((seed ^ CAND_SALT) & 0xFFFFFFFFFFFFFFFF)
    for i in range(min(k, F)):
        h = int(hash3(s, key, np.uint64(i)))
        j = i + h % (F - i)
        arr[i], arr[j] = arr[j], arr[i]
    return np.array(arr[:min(k, F)], dtype=np.int64)


def n_candidates(strategy, F: int) -> int:
    s = str(strategy).lower()
    if s in ("all", "none"):
        return F
    if s in ("sqrt", "auto"):
        return max(1, math.ceil(math.sqrt(F)))
    if s == "log2":
        return max(1, math.ceil(math.log2(F)))
    if s == "onethird":
        return max(1, math.ceil(F / 3))
    frac = float(s)
    if not 0 < frac <= 1:
        raise ValueError(f"feature_subset fraction must be in (0, 1], got {strategy}")
    return max(1, math.ceil(frac * F))


def pack_bits(B: np.ndarray) -> np.ndarray:
    """[N, F] {0,1} -> [N, ceil(F/64)] uint64 (feature f = bit f%64 of word f//64)."""
    B = np.asarray(B).astype(bool)
    n, F = B.shape
    W = max(1, (F + 63) // 64)
    out = np.zeros((n, W), dtype=np.uint64)
    for f in range(F):
        out[:, f // 64] |= B[:, f].astype(np.uint64) << np.uint64(f % 64)
    return out


def unpack_bits(Xw: np.ndarray, F: int) -> np.ndarray:
    Xw = np.asarray(Xw, dtype=np.uint64).reshape(len(Xw), -1)
    out = np.zeros((len(Xw), F), dtype=np.int64)
    for f in range(F):
        out[:, f] = ((Xw[:, f // 64] >> np.uint64(f % 64)) & np.uint64(1)).astype(np.int64)
    return out


def draw_features(numbers: np.ndarray, lags: int = 1) -> tuple[np.ndarray, np.ndarray, int]:
    """Draw rows -> (X bits [S, W], Y masks [S], F) for samples t = lags-1 .. N-2."""
    from ..data.draws import lag_features, mask_bits

    if lags == 1:
        m = mask_bits(numbers)
        return m[:-1].reshape(-1, 1).copy(), m[1:].copy(), 62
    X, Y = lag_features(numbers, lags)
    return pack_bits(X), pack_bits(Y)[:, 0].copy(), 62 * lags


class RandomForest:
    def __init__(self, n_trees: int = 100, max_depth: int = 8, min_samples_leaf: int = 1,
                 feature_subset="sqrt", bootstrap: bool = True, seed: int = 0, device: str = "auto"):
        if not 0 <= max_depth <= 14:
            raise ValueError("max_depth must be in [0, 14] (complete-array trees)")
        if n_trees < 1 or min_samples_leaf < 1:
            raise ValueError("n_trees and min_samples_leaf must be >= 1")
        self.n_trees, self.max_depth, self.min_samples_leaf = int(n_trees), int(max_depth), int(min_samples_leaf)
        self.feature_subset, self.bootstrap, self.seed, self.device = feature_subset, bool(bootstrap), int(seed), device
        self.nodes = (1 << (max_depth + 1)) - 1
        self.F = None
        self.feat = self.value = self.gain = self.cover = None
        self.backend_used = None

    # ------------------------------------------------------------------ fit
    def _backend(self) -> str:
        if self.device == "cpu":
            return "numpy"
        try:
            import torch

            if torch.cuda.is_available():
                return "hip"
        except Exception:  # noqa: BLE001
            pass
        if self.device == "cuda":
            raise RuntimeError("device=cuda requested but no GPU is available")
        return "numpy"

    def fit(self, X: np.ndarray, Y: np.ndarray, F: int, trees: range | None = None, group=None) -> "RandomForest":
        """X: [N, W] uint64 feature bits, Y: [N] uint64 target masks (bits 0..61), F features."""
        X = np.ascontiguousarray(np.asarray(X, dtype=np.uint64).reshape(len(X), -1))
        Y = np.ascontiguousarray(np.asarray(Y, dtype=np.uint64).reshape(-1))
        if F > 64 * X.shape[1] or F > 256:
            raise ValueError("F exceeds the packed feature words (max 256)")
        self.F = int(F)
        self.k = n_candidates(self.feature_subset, F)
        if trees is None:
            trees = range(self.n_trees)
            if group is not None:
                from ..parallel.dist import shard_range, DistInfo
                import torch.distributed as dist

                info = DistInfo(dist.get_rank(group), dist.get_world_size(group))
                a, b = shard_range(self.n_trees, info)
                trees = range(a, b)
        be = self._backend()
        self.backend_used = be
        if be == "hip":
            feat, value, gain, cover = self._fit_hip(X, Y, trees)
        else:
            feat, value, gain, cover = self._fit_numpy(X, Y, trees)
        if group is not None:
            feat, value, gain, cover = self._gather(group, trees, feat, value, gain, cover)
        self.feat, self.value, self.gain, self.cover = feat, value, gain, cover
        return self

    def _fit_numpy(self, X, Y, trees):
        from .forest_oracle import grow_forest_numpy

        return grow_forest_numpy(X, Y, self.F, list(trees), self.max_depth, self.k, self.min_samples_leaf,
                                 self.bootstrap, self.seed)

    def _fit_hip(self, X, Y, trees):
        import torch

        from ..ops import forest as K

        return K.fit(X, Y, self.F, trees.start, len(trees), self.max_depth, self.k, self.min_samples_leaf,
                     self.bootstrap, self.seed)

    def _gather(self, group, trees, feat, value, gain, cover):
        """C5: all-gather the packed per-rank tree arrays (tree ids are global, so order is fixed)."""
        import torch.distributed as dist

        parts = [None] * dist.get_world_size(group)
        dist.all_gather_object(parts, (trees.start, feat, value, gain, cover), group=group)
        parts.sort(key=lambda p: p[0])
        return tuple(np.concatenate([p[i] for p in parts]) for i in range(1, 5))

    # ------------------------------------------------------------------ predict
    def predict_proba(self, X: np.ndarray) -> np.ndarray:
        """[N, 62] mean leaf vector over trees (numpy traversal)."""
        X = np.asarray(X, dtype=np.uint64).reshape(len(X), -1)
        n = len(X)
        bits = unpack_bits(X, self.F)
        acc = np.zeros((n, 64), dtype=np.float64)
        rows = np.arange(n)
        for t in range(len(self.feat)):
            node = np.zeros(n, dtype=np.int64)
            for _ in range(self.max_depth + 1):
                f = self.feat[t][node]
                act = f >= 0
                if not act.any():
                    break
                b = bits[rows[act], f[act]]
                node[act] = 2 * node[act] + 1 + b
            acc += self.value[t][node]
        return (acc / max(len(self.feat), 1))[:, :62].astype(np.float32)

    def predict_proba_device(self, X, out_logit: bool = False):
        """Same on the GPU (K11): returns a [N, 64] fp32 device tensor."""
        from ..ops import forest as K

        return K.predict(X, self.feat, self.value, self.max_depth, out_logit=out_logit)

    # ------------------------------------------------------------------ persistence (T6 tree file)
    def meta(self) -> dict:
        return {"format": "euromillioner-forest-v1", "n_trees": len(self.feat), "max_depth": self.max_depth,
                "min_samples_leaf": self.min_samples_leaf, "feature_subset": str(self.feature_subset),
                "bootstrap": self.bootstrap, "seed": self.seed, "F": self.F, "k": self.k}

    def save(self, path: str) -> None:
        """``.npz`` of plain arrays + JSON meta (loadable with allow_pickle=False)."""
        np.savez(path, feat=self.feat, value=self.value, gain=self.gain, cover=self.cover,
                 meta=np.frombuffer(json.dumps(self.meta()).encode(), dtype=np.uint8))

    @classmethod
    def load(cls, path: str) -> "RandomForest":
        z = np.load(path, allow_pickle=False)
        meta = json.loads(bytes(z["meta"]).decode())
        if meta.get("format") != "euromillioner-forest-v1":
            raise ValueError("not a forest file")
        rf = cls(meta["n_trees"], meta["max_depth"], meta["min_samples_leaf"], meta["feature_subset"],
                 meta["bootstrap"], meta["seed"])
        rf.F, rf.k = meta["F"], meta["k"]
        rf.feat, rf.value, rf.gain, rf.cover = z["feat"], z["value"], z["gain"], z["cover"]
        return rf
