"""Property tests of the HIP tree engines against their numpy oracles over random small problems:
row counts from a handful (nodes that empty out, single-chunk levels) to a few thousand, random
depths, feature subsets, bootstrap on/off, lag windows (RF); random depth / eta / gamma /
objective (GBDT).  Both engines promise exact agreement (RF: identical trees, values and gains;
GBDT: identical splits, leaves to 1e-5)."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from euromillioner_amd.data.draws import DrawSet, multi_hot

pytestmark = pytest.mark.gpu


@settings(max_examples=12, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.integers(5, 4000), st.integers(1, 8), st.sampled_from(["sqrt", "log2", "all", "0.3"]), st.booleans(),
       st.sampled_from([1, 2]), st.integers(0, 1000), st.integers(1, 12))
def test_rf_hip_matches_oracle_random(n, depth, subset, boot, lags, seed, trees):
    from euromillioner_amd.models.forest import RandomForest, draw_features

    ds = DrawSet.synthetic(n=n + lags + 1, seed=seed, planted=0.7, calendar=False)
    X, Y, F = draw_features(ds.numbers, lags)
    kw = dict(n_trees=trees, max_depth=depth, feature_subset=subset, bootstrap=boot, seed=seed)
    gpu = RandomForest(device="cuda", **kw).fit(X, Y, F)
    assert gpu.backend_used == "hip"
    cpu = RandomForest(device="cpu", **kw).fit(X, Y, F)
    assert np.array_equal(gpu.feat, cpu.feat)
    live = gpu.feat > -2
    assert np.array_equal(gpu.value[live], cpu.value[live])
    assert np.array_equal(gpu.gain, cpu.gain)


@settings(max_examples=10, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.integers(8, 3000), st.integers(1, 4), st.sampled_from([0.3, 1.0]), st.sampled_from([0.0, 1.0]),
       st.sampled_from(["reg:logistic", "reg:squarederror"]), st.integers(0, 1000), st.integers(1, 3))
def test_gbdt_hip_matches_oracle_random(n, depth, eta, gamma, obj, seed, tasks):
    from euromillioner_amd.models import gbdt as G

    ds = DrawSet.synthetic(n=n + 1, seed=seed, planted=0.8, calendar=False)
    X = multi_hot(ds.numbers[:-1]).astype(np.float64)
    Y = multi_hot(ds.numbers[1:])[:, :tasks].astype(np.float64)
    kw = dict(nround=6, max_depth=depth, gamma=gamma, eta=eta, objective=obj,
              eval_metric="logloss" if obj == "reg:logistic" else "rmse")
    a = G.GBDT(backend="numpy", **kw).fit(X, Y)
    b = G.GBDT(backend="hip", **kw).fit(X, Y)
    assert np.array_equal(a.trees.status, b.trees.status)
    assert np.array_equal(a.trees.feat, b.trees.feat)
    assert np.allclose(a.trees.leaf, b.trees.leaf, atol=1e-5)
