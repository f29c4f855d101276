"""GBDT with XGBoost semantics: formulas, pruning, exact-vs-hist equivalence, persistence."""
import os

import numpy as np
import pytest

from euromillioner_amd.data.draws import DrawSet, featurize_raw, multi_hot
from euromillioner_amd.models import gbdt as G


def _ref_data(n=None):
    ds = DrawSet.synthetic(seed=1)
    raw = featurize_raw(ds).astype(float)
    return raw[:, 1:], (raw[:, 0] >= 5).astype(float)


def test_single_split_hand_computed():
    # 4 rows, one feature; logistic from margin 0: p = .5, g = p - y, h = .25
    X = np.array([[0.0], [0.0], [1.0], [1.0]])
    y = np.array([0.0, 0.0, 1.0, 1.0])
    m = G.GBDT(nround=1, max_depth=1, gamma=0.0, eta=1.0, min_child_weight=0.1, backend="numpy").fit(X, y)
    tr = m.trees
    # G_L = 1.0 (0.5+0.5), H_L = 0.5 ; G_R = -1.0, H_R = 0.5 ; G = 0, H = 1
    gain = 1.0 / 1.5 + 1.0 / 1.5 - 0.0
    assert tr.status[0, 0] == 1 and abs(tr.gain[0, 0] - gain) < 1e-6
    assert abs(tr.leaf[0, 1] - (-1.0 / 1.5)) < 1e-6 and abs(tr.leaf[0, 2] - (1.0 / 1.5)) < 1e-6
    assert tr.split_value[0, 0] == 0.5


def test_gamma_prunes_weak_split():
    X = np.array([[0.0], [0.0], [1.0], [1.0]])
    y = np.array([0.0, 0.0, 1.0, 1.0])
    m = G.GBDT(nround=1, max_depth=1, gamma=2.0, min_child_weight=0.1, backend="numpy").fit(X, y)  # gain 1.33 < gamma
    assert m.trees.status[0, 0] == 2 and (m.trees.status[0, 1:] == 0).all()


def test_min_child_weight_blocks_split():
    X = np.array([[0.0], [1.0], [1.0], [1.0]])
    y = np.array([1.0, 0.0, 0.0, 0.0])
    m = G.GBDT(nround=1, max_depth=1, gamma=0.0, min_child_weight=0.5, backend="numpy").fit(X, y)
    assert m.trees.status[0, 0] == 2  # left child hessian 0.25 < 0.5


def test_logistic_rejects_out_of_range_labels():
    X, _ = _ref_data()
    dow = featurize_raw(DrawSet.synthetic(seed=1))[:, 0].astype(float)
    with pytest.raises(ValueError, match=r"label must be in \[0,1\]"):
        G.GBDT(nround=1, backend="numpy").fit(X, dow)  # the reference's label_column=0 (defect D-d)


def test_hist_equals_exact_first_split():
    X, y = _ref_data()
    g = np.full(len(y), 0.5) - y
    h = np.full(len(y), 0.25)
    cuts = G.make_cuts(X, 256)
    bins = G.apply_bins(X, cuts)
    nb = max(len(c) for c in cuts) + 1
    hg = np.zeros((X.shape[1], nb))
    hh = np.zeros_like(hg)
    for f in range(X.shape[1]):
        hg[f] = np.bincount(bins[:, f], weights=g, minlength=nb)
        hh[f] = np.bincount(bins[:, f], weights=h, minlength=nb)
    gain, f, b, _, _ = G._best_split_hist(hg, hh, g.sum(), h.sum(), 1.0, 1.0)
    ex = [G.exact_greedy_split(X[:, k], g, h, 1.0, 1.0) for k in range(X.shape[1])]
    best_f = int(np.argmax([e[0] for e in ex]))
    assert best_f == f
    assert abs(ex[f][0] - gain) < 1e-9 and ex[f][1] == cuts[f][b]


def test_reference_config_trains_and_predicts():
    X, y = _ref_data()
    n = int(0.7 * len(y))
    m = G.GBDT.from_params({"booster": "gbtree", "eta": 1.0, "max_depth": 3, "objective": "reg:logistic",
                            "subsample": 1, "gamma": 1.0, "eval_metric": "logloss"}, nround=30, backend="numpy")
    m.fit(X[:n], y[:n], evals={"train": (X[:n], y[:n]), "test": (X[n:], y[n:])})
    assert len(m.history) == 30
    assert m.history[-1]["train"] < m.history[0]["train"]
    p = m.predict(X[:n])
    assert p.dtype == np.float32 and p.shape == (n, 1)
    # cpu_predictor traversal on raw values == margins accumulated during training
    assert np.allclose(G.transform(m.objective, m.predict_margin(X[:n])), p, atol=1e-6)


def test_multi_task_next_draw():
    ds = DrawSet.synthetic(n=3000, seed=4, planted=0.9, calendar=False)
    X = multi_hot(ds.numbers[:-1])
    Y = multi_hot(ds.numbers[1:])
    m = G.GBDT(nround=10, max_depth=3, gamma=1.0, eta=0.5, backend="numpy").fit(X[:2000], Y[:2000])
    P = m.predict(X[2000:])
    assert P.shape == (len(X) - 2000, 62)
    from euromillioner_amd import metrics as M

    met = M.draw_metrics(np.log(P / (1 - P)), Y[2000:])
    assert met["acc"] > 0.93


def test_json_roundtrip(tmp_path):
    X, y = _ref_data()
    m = G.GBDT(nround=5, backend="numpy").fit(X, y)
    p = tmp_path / "m.json"
    m.save(str(p))
    m2 = G.GBDT.load(str(p))
    assert np.array_equal(m.predict(X), m2.predict(X))


def _multi_data(n=700, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 6))
    y = (X[:, 0] > 0).astype(np.int64) + 2 * (X[:, 1] > 0.4) + (X[:, 2] > 1.2)
    return X, np.minimum(y, 3).astype(np.float64)


@pytest.mark.parametrize("obj", ["multi:softprob", "multi:softmax"])
def test_multiclass_softmax_learns(obj, tmp_path):
    X, y = _multi_data()
    m = G.GBDT(objective=obj, nround=25, eta=0.3, gamma=0.0, backend="numpy").fit(
        X[:500], y[:500], evals={"test": (X[500:], y[500:])})
    assert m.num_class == 4 and m.n_tasks == 4 and m.eval_metric == "mlogloss"
    assert m.history[-1]["test"] < 0.5 * m.history[0]["test"]
    p = m.predict(X[500:])
    if obj == "multi:softprob":
        assert p.shape == (200, 4) and np.allclose(p.sum(1), 1.0, atol=1e-5)
        p = np.argmax(p, 1)
    assert np.mean(p == y[500:]) > 0.85
    m.save(str(tmp_path / "m.json"))
    m2 = G.GBDT.load(str(tmp_path / "m.json"))
    assert m2.num_class == 4 and np.array_equal(m2.predict(X[500:]), m.predict(X[500:]))


def test_multiclass_first_round_gradients_by_hand():
    """Round-0 margins are base_score for every class -> p = 1/K, g = 1/K - y, h = 2/K (1 - 1/K)."""
    y1 = np.eye(3)[[0, 2, 1]].astype(np.float32)
    g, h = G.gradients("multi:softprob", np.full((3, 3), 0.5, np.float32), y1)
    assert np.allclose(g, 1 / 3 - y1) and np.allclose(h, 2 / 3 * (2 / 3))


def test_multiclass_rejects_bad_labels():
    X, y = _multi_data(50)
    with pytest.raises(ValueError):
        G.GBDT(objective="multi:softprob", nround=1, backend="numpy").fit(X, y + 0.5)
    with pytest.raises(ValueError):
        G.GBDT(objective="multi:softprob", num_class=2, nround=1, backend="numpy").fit(X, y)


def test_multiclass_metrics():
    from euromillioner_amd import metrics as M

    p = np.array([[0.7, 0.2, 0.1], [0.1, 0.1, 0.8]])
    assert abs(M.mlogloss(np.array([0, 1]), p) - (-(np.log(0.7) + np.log(0.1)) / 2)) < 1e-12
    assert M.merror(np.array([0, 1]), p) == 0.5
    assert M.merror(np.eye(3)[[0, 2]], p) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("obj", ["multi:softprob", "multi:softmax"])
def test_hip_multiclass_matches_oracle(obj):
    X, y = _multi_data(3000, seed=2)
    kw = dict(objective=obj, nround=15, eta=0.3, gamma=0.0, max_depth=3)
    a = G.GBDT(backend="numpy", **kw).fit(X[:2000], y[:2000], evals={"test": (X[2000:], y[2000:])})
    b = G.GBDT(backend="hip", **kw).fit(X[:2000], y[:2000], evals={"test": (X[2000:], y[2000:])})
    assert b.backend_used == "hip"
    assert np.array_equal(a.trees.feat, b.trees.feat) and np.array_equal(a.trees.sbin, b.trees.sbin)
    assert np.allclose(a.trees.leaf, b.trees.leaf, atol=1e-4)
    assert np.allclose(a.predict(X[2000:]), b.predict(X[2000:], backend="hip"), atol=1e-4)
    assert abs(a.history[-1]["test"] - b.history[-1]["test"]) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("obj", ["reg:logistic", "reg:squarederror"])
def test_hip_engine_matches_oracle(obj):
    X, y = _ref_data()
    n = int(0.7 * len(y))
    kw = dict(nround=40, max_depth=3, gamma=1.0, eta=1.0 if obj == "reg:logistic" else 0.3, objective=obj,
              eval_metric="logloss" if obj == "reg:logistic" else "rmse")
    a = G.GBDT(backend="numpy", **kw).fit(X[:n], y[:n], evals={"test": (X[n:], y[n:])})
    b = G.GBDT(backend="hip", **kw).fit(X[:n], y[:n], evals={"test": (X[n:], y[n:])})
    assert np.array_equal(a.trees.status, b.trees.status)
    assert np.array_equal(a.trees.feat, b.trees.feat)
    assert np.allclose(a.trees.leaf, b.trees.leaf, atol=1e-5)
    assert np.allclose(a.predict(X[n:]), b.predict(X[n:], backend="hip"), atol=1e-5)
    assert abs(a.history[-1]["test"] - b.history[-1]["test"]) < 1e-4


@pytest.mark.gpu
def test_hip_engine_multitask():
    ds = DrawSet.synthetic(n=20000, seed=4, planted=0.9, calendar=False)
    X = multi_hot(ds.numbers[:-1])
    Y = multi_hot(ds.numbers[1:])
    a = G.GBDT(nround=8, eta=0.5, backend="numpy").fit(X[:15000], Y[:15000])
    b = G.GBDT(nround=8, eta=0.5, backend="hip").fit(X[:15000], Y[:15000])
    assert np.array_equal(a.trees.feat, b.trees.feat)
    assert np.allclose(a.predict(X[15000:]), b.predict(X[15000:], backend="hip"), atol=1e-5)


@pytest.mark.gpu
def test_hip_dp_primitives_match_single_call():
    """The data-parallel HIP path (per-level hist -> all-reduce -> split) on a 1-rank RCCL group
    reproduces the fused multi-round driver exactly (C4 plumbing on one GPU)."""
    import socket

    import torch
    import torch.distributed as dist

    from euromillioner_amd import config as C
    from euromillioner_amd.data.draws import DrawSet
    from euromillioner_amd.models.gbdt import GBDT
    from euromillioner_amd.pipeline import gbdt_dataset

    ds = DrawSet.synthetic(n=900, seed=8, planted=0.6, calendar=True)
    X, Y, _ = gbdt_dataset(ds, C.RunConfig())
    Y = Y[:, :5]
    kw = dict(eta=0.7, max_depth=3, gamma=0.5, min_child_weight=0.5, nround=12, backend="hip")
    ref = GBDT(**kw).fit(X[:600], Y[:600], evals={"test": (X[600:], Y[600:])})
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        dp = GBDT(**kw).fit(X[:600], Y[:600], evals={"test": (X[600:], Y[600:])}, group=dist.group.WORLD)
    finally:
        dist.destroy_process_group()
    assert np.array_equal(dp.trees.feat, ref.trees.feat) and np.array_equal(dp.trees.sbin, ref.trees.sbin)
    assert np.array_equal(dp.trees.leaf, ref.trees.leaf)
    assert np.allclose([h["test"] for h in dp.history], [h["test"] for h in ref.history], rtol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("obj", ["reg:logistic", "reg:squarederror"])
def test_hip_fused_round_bit_identical(obj):
    """The fused round (partition inside the histogram pass, prune/leaves in the last split, the update
    of round r - 1 -- last partition, margins, eval predictions, round r's g / h -- inside round r's
    level-0 histogram pass) and the separate launches give bit-identical trees, margins and predictions,
    and the same metric history to float rounding (the metric terms are summed in another grouping)."""
    from euromillioner_amd import config as C
    from euromillioner_amd.pipeline import gbdt_dataset

    ds = DrawSet.synthetic(n=None, seed=3, planted=0.5)
    X, Y, _ = gbdt_dataset(ds, C.RunConfig())
    m = int(0.7 * len(X))
    kw = dict(eta=1.0 if obj == "reg:logistic" else 0.3, max_depth=3, gamma=1.0, nround=60, objective=obj,
              eval_metric="logloss" if obj == "reg:logistic" else "rmse", subsample=0.8, backend="hip")
    ev = {"test": (X[m:], Y[m:])}
    fits = {}
    for name in ("fused", "separate", "presplit"):
        g = G.GBDT(**kw)
        g.separate_launches = name == "separate"
        g.presplit_levels = name == "presplit"  # level L's split inside level L + 1's histogram pass
        fits[name] = g.fit(X[:m], Y[:m], evals=ev)
    a, b = fits["fused"], fits["separate"]
    for k in ("status", "feat", "sbin", "leaf", "gain", "cover"):
        assert np.array_equal(getattr(a.trees, k), getattr(b.trees, k)), k
        assert np.array_equal(getattr(fits["presplit"].trees, k), getattr(b.trees, k)), k
    # (the fused rounds sum the per-round metric terms grouped by histogram chunk, the separate launches by
    # update block: the same terms, summed in another order)
    assert len(a.history) == len(b.history)
    for ha, hb in zip(a.history, b.history):
        assert ha.keys() == hb.keys() and all(abs(ha[k] - hb[k]) <= 1e-6 * max(1.0, abs(hb[k])) for k in ha), (ha, hb)
    assert np.array_equal(a.predict(X[m:], backend="hip"), b.predict(X[m:], backend="hip"))


def test_native_hist_plan_bounds():
    """The GBDT device planner (host C++, runs without a GPU): small shapes plan, the per-chunk
    partial buffer stays under its 1 GiB cap for deep 256-bin trees, and impossible shapes are
    refused (-1) instead of asking for terabytes."""
    import numpy as np
    import pytest

    from euromillioner_amd.ops import _native as N

    if not N.available():
        pytest.skip("native library not built")
    from euromillioner_amd.models import gbdt_hip  # noqa: F401  (registers the signatures)

    def need(n, T, F, nb, D):
        off = np.concatenate([[0], np.cumsum([nb] * F)]).astype(np.int32)
        return N.query("em_gbdt_partial_doubles", n, T, F, off.ctypes.data, D)

    assert 0 < need(928, 62, 66, 3, 3) <= 1 << 27
    assert 0 < need(183500, 62, 66, 7, 3) <= 1 << 27
    assert 0 < need(100000, 62, 66, 256, 6) <= 1 << 27
    assert need(100000, 62, 66, 256, 12) == -1
    off = np.array([0, 2, 300], dtype=np.int32)  # a feature with 298 bins is not supported
    assert N.query("em_gbdt_partial_doubles", 1000, 1, 2, off.ctypes.data, 3) == -1


@pytest.mark.gpu
def test_hip_engine_deep_many_bins_matches_oracle():
    """Continuous features (256 bins each) on depth-6 trees: the device planner tiles features and
    nodes and stages rows in several LDS pieces per chunk; trees still match the numpy oracle."""
    rng = np.random.default_rng(7)
    n = 6000
    X = rng.normal(size=(n, 12))
    y = ((X[:, 0] + 0.5 * X[:, 3] * X[:, 5] + 0.3 * rng.normal(size=n)) > 0).astype(np.float64)
    kw = dict(nround=6, max_depth=6, eta=0.5, gamma=0.0, min_child_weight=0.5)
    a = G.GBDT(backend="numpy", **kw).fit(X[:4500], y[:4500], evals={"test": (X[4500:], y[4500:])})
    b = G.GBDT(backend="hip", **kw).fit(X[:4500], y[:4500], evals={"test": (X[4500:], y[4500:])})
    assert b.backend_used == "hip"
    assert np.array_equal(a.trees.status, b.trees.status)
    assert np.array_equal(a.trees.feat, b.trees.feat) and np.array_equal(a.trees.sbin, b.trees.sbin)
    assert np.allclose(a.trees.leaf, b.trees.leaf, atol=1e-5)
    assert abs(a.history[-1]["test"] - b.history[-1]["test"]) < 1e-5


# ----------------------------------------------------------------------------- fixed-point histograms
def test_quant_bits_rule():
    assert G.quant_bits("reg:logistic", 928) == 0  # reference config: exact fp64 sums
    assert G.quant_bits("reg:logistic", 183500) == 61 - 18  # 2^17 < 183500 < 2^18
    assert G.quant_bits("multi:softprob", 40000) == 61 - 16
    assert G.quant_bits("reg:squarederror", 183500) == 0  # unbounded g: always exact
    assert G.quant_bits("reg:logistic", 183500, distributed=True) == 0  # DP all-reduces fp64
    assert G.quant_bits("reg:logistic", 183500, mode="exact") == 0
    assert G.quant_bits("reg:logistic", 500, mode="quant") == 61 - 9
    with pytest.raises(ValueError):
        G.quant_bits("reg:logistic", 10, mode="fast")


def test_int_hist_is_exact():
    """The oracle's integer histogram (two float64 GEMMs of 26-bit halves) equals exact integer sums
    at the largest magnitudes quant_bits allows."""
    rng = np.random.default_rng(0)
    n, C, K = 5000, 40, 7
    s = G.quant_bits("reg:logistic", n, mode="quant")
    Z = rng.integers(-(1 << s), (1 << s) + 1, size=(n, K), dtype=np.int64)
    Z[:, 0] = 1 << s  # worst case: every row at the bound
    onehot = np.zeros((n, C))
    onehot[np.arange(n), rng.integers(0, C, n)] = 1.0
    onehot[:, 0] = 1.0
    exact = onehot.astype(np.int64).T @ Z  # int64 matmul: exact (|sums| < 2^61)
    assert np.array_equal(G._int_hist(onehot, Z), exact)


@pytest.mark.parametrize("obj", ["reg:logistic", "multi:softprob"])
def test_quantised_oracle_tracks_exact(obj):
    """hist_mode="quant" changes only the rounding of the histogram sums (2^-s ~ 1e-13 here): the
    trees of the first rounds are the exact-mode trees and the losses agree to ~1e-9."""
    if obj == "reg:logistic":
        X, y = _ref_data()
    else:
        X, y = _multi_data(1500, seed=3)
    n = int(0.7 * len(y))
    kw = dict(objective=obj, nround=6, max_depth=3, eta=0.5, gamma=0.0, backend="numpy")
    a = G.GBDT(hist_mode="exact", **kw).fit(X[:n], y[:n], evals={"test": (X[n:], y[n:])})
    b = G.GBDT(hist_mode="quant", **kw).fit(X[:n], y[:n], evals={"test": (X[n:], y[n:])})
    assert a.quant_bits_used == 0 and b.quant_bits_used > 40
    assert np.array_equal(a.trees.feat, b.trees.feat) and np.array_equal(a.trees.sbin, b.trees.sbin)
    assert np.allclose(a.trees.leaf, b.trees.leaf, rtol=1e-6, atol=1e-9)
    assert abs(a.history[-1]["test"] - b.history[-1]["test"]) < 1e-6


def test_quantised_sums_are_order_free():
    """Permuting the rows leaves every fixed-point tree bit-identical (integer sums), which is what
    lets the device accumulate them with order-free atomics."""
    X, y = _ref_data()
    kw = dict(nround=4, max_depth=3, eta=0.5, gamma=0.0, backend="numpy", hist_mode="quant")
    perm = np.random.default_rng(1).permutation(len(y))
    a = G.GBDT(**kw).fit(X, y)
    b = G.GBDT(**kw).fit(X[perm], y[perm])
    assert np.array_equal(a.trees.feat, b.trees.feat) and np.array_equal(a.trees.sbin, b.trees.sbin)
    assert np.array_equal(a.trees.leaf, b.trees.leaf)


def _saturating_data(n=3000, seed=5):
    """Labels a function of one feature; fitted from base_score = 1 - 2^-53 (SAT_KW), i.e. a margin of
    ~36.7 where float32 p == 1 and every row sits at the logistic hessian floor (1e-16)."""
    rng = np.random.default_rng(seed)
    X = rng.integers(0, 8, size=(n, 4)).astype(float)
    return X, (X[:, 0] >= 4).astype(float)


SAT_KW = dict(nround=3, max_depth=3, eta=1.0, gamma=0.0, min_child_weight=0.0, reg_lambda=0.0,
              base_score=1 - 2 ** -53)


def test_quantised_hessian_floor_keeps_nodes_positive():
    """with fixed-point sums a row at the 1e-16 hessian floor quantises to q = 0 at
    s < 53, so a node of saturated rows had H == 0 where the exact form keeps H > 0, and with
    min_child_weight = reg_lambda = 0 its gain and leaf were 0/0.  A positive h now quantises to at
    least one quantum (oracle and csrc/gbdt.hip quantise_h): every leaf stays finite."""
    X, y = _saturating_data()
    m = G.GBDT(hist_mode="quant", backend="numpy", **SAT_KW).fit(X, y)  # (without the fix: -inf leaves)
    assert m.quant_bits_used > 0
    assert np.isfinite(m.trees.leaf).all() and np.isfinite(m.trees.gain).all()
    assert (m.trees.cover[m.trees.status != 0] > 0).all()
    assert np.isfinite(m.predict(X)).all()
    q = G._quantise_h(np.array([1e-16, 0.0, 0.25], np.float32), 40)
    assert q.tolist() == [1, 0, 1 << 38]


def test_segment_cumsum_has_no_cross_feature_intermediate():
    """the fixed-point left sums are per feature segment, so no int64 intermediate grows
    with the feature count: 62 one-hot features whose cells all sit near the per-node bound (a
    cumsum over all of them would exceed 2^63) give the exact per-feature left sums."""
    F, big = 62, (1 << 60) // 2
    off = np.arange(0, 2 * F + 1, 2)
    hist = np.full((2 * F, 3), big, dtype=np.int64)
    got = G._segment_cumsum(hist, off)
    want = np.tile(np.array([[big], [2 * big]], dtype=np.int64), (F, 3))
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_hip_quantised_saturated_matches_oracle():
    """The device's quantise_h (fixed-point hessians never round to 0) reproduces the oracle on the
    saturating case: identical trees, finite leaves."""
    X, y = _saturating_data()
    a = G.GBDT(backend="numpy", hist_mode="quant", **SAT_KW).fit(X, y)
    b = G.GBDT(backend="hip", hist_mode="quant", **SAT_KW).fit(X, y)
    assert np.array_equal(a.trees.status, b.trees.status) and np.array_equal(a.trees.feat, b.trees.feat)
    assert np.array_equal(a.trees.sbin, b.trees.sbin)
    assert np.isfinite(b.trees.leaf).all()
    assert np.allclose(a.trees.leaf, b.trees.leaf, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("obj", ["reg:logistic", "multi:softprob"])
def test_hip_quantised_matches_oracle(obj):
    """Fixed-point device histograms (LDS int64 atomics) == the oracle's quantised mode, bit for bit
    in the tree structure, on a multi-chunk, multi-piece problem."""
    ds = DrawSet.synthetic(n=40001, seed=5, planted=0.9, calendar=False)
    X = multi_hot(ds.numbers[:-1])
    if obj == "reg:logistic":
        Y = multi_hot(ds.numbers[1:])[:, :9]
    else:
        Y = (ds.numbers[1:, 0] % 5).astype(np.float64)
    kw = dict(objective=obj, nround=5, eta=0.5, max_depth=3, gamma=0.0, hist_mode="quant")
    a = G.GBDT(backend="numpy", **kw).fit(X[:36000], Y[:36000], evals={"test": (X[36000:], Y[36000:])})
    b = G.GBDT(backend="hip", **kw).fit(X[:36000], Y[:36000], evals={"test": (X[36000:], Y[36000:])})
    assert b.backend_used == "hip" and b.quant_bits_used == a.quant_bits_used > 0
    assert np.array_equal(a.trees.status, b.trees.status)
    assert np.array_equal(a.trees.feat, b.trees.feat) and np.array_equal(a.trees.sbin, b.trees.sbin)
    assert np.allclose(a.trees.leaf, b.trees.leaf, atol=1e-5)
    assert abs(a.history[-1]["test"] - b.history[-1]["test"]) < 1e-5


@pytest.mark.gpu
def test_hip_quantised_mixed_features_match_oracle():
    """The reference feature set (63 one-hot lag features + 3 calendar features with 12-196 bins) at
    a size where both sparse passes run (row-per-lane one-hot kernel + lane-per-feature calendar
    kernel, several chunks): trees bit-identical to the oracle's quantised mode."""
    from euromillioner_amd import config as C
    from euromillioner_amd.pipeline import gbdt_dataset

    ds = DrawSet.synthetic(n=30001, seed=6, planted=0.5)
    X, Y, _ = gbdt_dataset(ds, C.RunConfig())
    Y = Y[:, :6]
    m = 24000
    kw = dict(nround=4, eta=1.0, max_depth=3, gamma=1.0, hist_mode="quant")
    a = G.GBDT(backend="numpy", **kw).fit(X[:m], Y[:m], evals={"test": (X[m:], Y[m:])})
    b = G.GBDT(backend="hip", **kw).fit(X[:m], Y[:m], evals={"test": (X[m:], Y[m:])})
    assert b.backend_used == "hip" and b.quant_bits_used == a.quant_bits_used > 0
    assert np.array_equal(a.trees.status, b.trees.status)
    assert np.array_equal(a.trees.feat, b.trees.feat) and np.array_equal(a.trees.sbin, b.trees.sbin)
    assert np.allclose(a.trees.leaf, b.trees.leaf, atol=1e-5)


@pytest.mark.gpu
def test_hip_quantised_dense_form_matches_oracle():
    """Continuous features only (no one-hot block): the fixed-point form runs the lane-per-feature
    kernel over all features (staged bin rows, one shared LDS copy, derived bin 0); depth-6 trees
    over 256-bin features stay bit-identical to the oracle's quantised mode."""
    rng = np.random.default_rng(11)
    n = 6000
    X = rng.normal(size=(n, 12))
    y = ((X[:, 0] + 0.5 * X[:, 3] * X[:, 5] + 0.3 * rng.normal(size=n)) > 0).astype(np.float64)
    kw = dict(nround=4, max_depth=6, eta=0.5, gamma=0.0, min_child_weight=0.5, hist_mode="quant")
    a = G.GBDT(backend="numpy", **kw).fit(X[:4500], y[:4500], evals={"test": (X[4500:], y[4500:])})
    b = G.GBDT(backend="hip", **kw).fit(X[:4500], y[:4500], evals={"test": (X[4500:], y[4500:])})
    assert b.backend_used == "hip" and b.quant_bits_used == a.quant_bits_used > 0
    assert np.array_equal(a.trees.status, b.trees.status)
    assert np.array_equal(a.trees.feat, b.trees.feat) and np.array_equal(a.trees.sbin, b.trees.sbin)
    assert np.allclose(a.trees.leaf, b.trees.leaf, atol=1e-5)
