"""numpy oracle for the random forest engine (``csrc/forest.hip``): the same level-wise
algorithm with the same hashes and the same double-precision gain expression, so the
GPU forest can be compared array-for-array (CPU backend and test reference).  The forest is
declared, never built, by the reference (``/root/reference/pom.xml:56-61``)."""
from __future__ import annotations

import numpy as np

from .forest import candidates, poisson_weights, unpack_bits


def grow_forest_numpy(X, Y, F, trees, max_depth, k, min_leaf, bootstrap, seed):
    nodes = (1 << (max_depth + 1)) - 1
    T = len(trees)
    feat = np.full((T, nodes), -2, dtype=np.int16)
    value = np.zeros((T, nodes, 64), dtype=np.float32)
    gain = np.zeros((T, nodes), dtype=np.float64)
    cover = np.zeros((T, nodes), dtype=np.float32)
    N = len(X)
    xb = unpack_bits(X, F)  # [N, F] int64
    yb = unpack_bits(Y.reshape(-1, 1), 62)  # [N, 62]
    for ti, t in enumerate(trees):
        w = poisson_weights(seed, t, N) if bootstrap else np.ones(N, dtype=np.int64)
        frontier = {0: np.nonzero(w > 0)[0]}
        for level in range(max_depth + 1):
            nxt = {}
            for node, rows in frontier.items():
                wr = w[rows]
                n = int(wr.sum())
                S = (yb[rows] * wr[:, None]).sum(0)  # [62] exact ints
                cover[ti, node] = np.float32(n)
                if n > 0:
                    value[ti, node, :62] = (S.astype(np.float64) / float(n)).astype(np.float32)
                f_best, g_best = -1, 0.0
                if level < max_depth and n >= 2 * min_leaf and n > 0:
                    xr = xb[rows]
                    cnt = (xr * wr[:, None]).sum(0)  # [F]
                    hist = xr.T @ (yb[rows] * wr[:, None])  # [F, 62] exact (int64)
                    s2 = int((S * S).sum())
                    for f in sorted(int(c) for c in candidates(seed, t, node, F, k)):
                        nR = int(cnt[f])
                        nL = n - nR
                        if nL < min_leaf or nR < min_leaf or nL == 0 or nR == 0:
                            continue
                        SR = hist[f]
                        SL = S - SR
                        aL, aR = int((SL * SL).sum()), int((SR * SR).sum())
                        g = float(aL) / float(nL) + float(aR) / float(nR) - float(s2) / float(n)
                        if f_best < 0 or g > g_best:
                            f_best, g_best = f, g
                    if f_best >= 0 and not (g_best > 1e-9 * (1.0 + g_best)):
                        f_best = -1
                    if f_best >= 0 and not (g_best > 0.0):
                        f_best = -1
                feat[ti, node] = f_best
                gain[ti, node] = g_best if f_best >= 0 else 0.0
                if f_best >= 0:
                    right = xb[rows, f_best] == 1
                    nxt[2 * node + 1] = rows[~right]
                    nxt[2 * node + 2] = rows[right]
            frontier = nxt
    return feat, value, gain, cover
