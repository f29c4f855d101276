"""External parity pin for the random-forest engine: the numpy oracle (models/forest_oracle.py), which
the HIP forest (csrc/forest.hip) reproduces bit for bit on the GPU (tests/test_forest.py GPU cases),
against scikit-learn's DecisionTreeRegressor on the same bootstrap sample.

Why these settings are the same learner (reference intent: Spark MLlib RF, /root/reference/pom.xml:56-61,
README.md:6): with ``criterion="squared_error"`` and multi-output {0,1} targets, sklearn's weighted
impurity decrease n_p*imp_p - n_L*imp_L - n_R*imp_R, times the 62 outputs, equals the oracle's gain
SL²/nL + SR²/nR - S²/n (for binary y, sum(w y²) = sum(w y) = S, so the linear terms cancel).  The Poisson
bootstrap weights go to sklearn as ``sample_weight`` on the rows with weight > 0.  Binary features split at
0.5, so sklearn's left child is the oracle's x = 0 child.  Where two features give the same best gain the
two learners may break the tie differently (oracle: lowest feature index; sklearn: its own feature order):
such nodes are counted and reported, and their subtrees are not compared."""
import numpy as np
import pytest

from euromillioner_amd.data.draws import DrawSet
from euromillioner_amd.models import forest as FO
from euromillioner_amd.models.forest import draw_features
from euromillioner_amd.models.forest_oracle import grow_forest_numpy

sk_tree = pytest.importorskip("sklearn.tree")


def _oracle_gains(xb, yb, w, rows, F):
    """Every feature's gain at a node (the oracle's expression), for the tie census."""
    wr = w[rows]
    n = int(wr.sum())
    S = (yb[rows] * wr[:, None]).sum(0)
    xr = xb[rows]
    cnt = (xr * wr[:, None]).sum(0)
    hist = xr.T @ (yb[rows] * wr[:, None])
    s2 = int((S * S).sum())
    g = np.full(F, -np.inf)
    for f in range(F):
        nR = int(cnt[f])
        nL = n - nR
        if nL < 1 or nR < 1:
            continue
        SR = hist[f]
        SL = S - SR
        g[f] = float(int((SL * SL).sum())) / nL + float(int((SR * SR).sum())) / nR - float(s2) / n
    return g


@pytest.mark.parametrize("depth,seed", [(4, 3), (6, 11)])
def test_oracle_tree_matches_sklearn(depth, seed, capsys):
    ds = DrawSet.synthetic(n=60_001, seed=seed, planted=0.8, calendar=False)
    X, Y, F = draw_features(ds.numbers)
    N = len(X)
    assert N >= 50_000
    feat, value, gain, cover = grow_forest_numpy(X, Y, F, [0], depth, F, 1, True, seed)
    feat, value, gain = feat[0], value[0], gain[0]

    xb = FO.unpack_bits(X, F)
    yb = FO.unpack_bits(Y.reshape(-1, 1), 62)
    w = FO.poisson_weights(seed, 0, N)
    boot = np.nonzero(w > 0)[0]
    sk = sk_tree.DecisionTreeRegressor(criterion="squared_error", max_depth=depth, max_features=None,
                                       min_samples_leaf=1, min_samples_split=2, random_state=0)
    sk.fit(xb[boot].astype(np.float64), yb[boot].astype(np.float64), sample_weight=w[boot].astype(np.float64))
    t = sk.tree_

    # walk both trees from the root; oracle node i <-> sklearn node j
    compared, tied_nodes = 0, set()
    stack = [(0, 0, boot)]
    while stack:
        i, j, rows = stack.pop()
        o_leaf = feat[i] < 0
        s_leaf = t.children_left[j] == -1
        if o_leaf or s_leaf:
            if o_leaf != s_leaf:
                # the only legitimate disagreement: a node the oracle keeps as a leaf because its best gain is
                # zero (sklearn may split on a zero-improvement candidate); anything else is a failure
                g = _oracle_gains(xb, yb, w, rows, F)
                assert o_leaf and not (g.max() > 1e-9 * (1.0 + abs(g.max()))), (i, j, g.max())
            continue
        g = _oracle_gains(xb, yb, w, rows, F)
        best = g.max()
        tied = np.nonzero(np.abs(g - best) <= 1e-12 * max(1.0, abs(best)))[0]
        fs = int(t.feature[j])
        if len(tied) > 1:
            tied_nodes.add(i)
            assert fs in tied, (i, fs, tied)
            continue
        compared += 1
        assert fs == int(feat[i]), (i, fs, int(feat[i]))
        # gain: oracle expression == 62 x sklearn's weighted impurity decrease
        nL, nR = t.weighted_n_node_samples[t.children_left[j]], t.weighted_n_node_samples[t.children_right[j]]
        dec = (t.weighted_n_node_samples[j] * t.impurity[j] - nL * t.impurity[t.children_left[j]]
               - nR * t.impurity[t.children_right[j]]) * 62
        assert abs(dec - gain[i]) <= 1e-6 * max(1.0, abs(gain[i])), (i, dec, gain[i])
        right = xb[rows, fs] == 1
        stack.append((2 * i + 1, int(t.children_left[j]), rows[~right]))
        stack.append((2 * i + 2, int(t.children_right[j]), rows[right]))

    # per-row predictions (any row, not only the bootstrap sample) for rows whose oracle path avoids the
    # tied nodes
    def oracle_predict(xrow):
        i = 0
        while feat[i] >= 0:
            if i in tied_nodes:
                return None
            i = 2 * i + 2 if xrow[feat[i]] == 1 else 2 * i + 1
        return value[i, :62]

    rng = np.random.default_rng(0)
    sample = rng.choice(N, size=6000, replace=False)
    got = [(r, oracle_predict(xb[r])) for r in sample]
    got = [(r, p) for r, p in got if p is not None]
    assert len(got) >= 3000
    rows_cmp = np.array([r for r, _ in got])
    po = np.stack([p for _, p in got])
    pred_sk = sk.predict(xb[rows_cmp].astype(np.float64))
    assert np.max(np.abs(po - pred_sk)) <= 1e-6
    ties = len(tied_nodes)
    with capsys.disabled():
        print(f"\n[rf-sklearn parity] depth {depth}, {N} rows ({len(boot)} in the bootstrap sample): "
              f"{compared} internal nodes matched (feature + gain), {ties} nodes with tied best gains skipped")
    assert compared >= 2 ** min(depth, 4) - 1
