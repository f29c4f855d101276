"""Random forest: numpy oracle semantics (CPU) and HIP engine == oracle (GPU)."""
import numpy as np
import pytest

from euromillioner_amd.data.draws import DrawSet, multi_hot
from euromillioner_amd.models import forest as FO
from euromillioner_amd.models.forest import RandomForest, draw_features


@pytest.fixture(scope="module")
def draws():
    ds = DrawSet.synthetic(n=2500, seed=4, planted=0.8, calendar=False)
    X, Y, F = draw_features(ds.numbers)
    return ds, X, Y, F


def test_pack_unpack_roundtrip():
    rng = np.random.default_rng(0)
    B = rng.integers(0, 2, size=(50, 130))
    assert np.array_equal(FO.unpack_bits(FO.pack_bits(B), 130), B)


def test_poisson_weights_distribution():
    w = FO.poisson_weights(7, 3, 200000)
    assert abs(w.mean() - 1.0) < 0.01
    assert abs((w == 0).mean() - np.exp(-1)) < 0.005
    assert np.array_equal(w, FO.poisson_weights(7, 3, 200000))
    assert not np.array_equal(w, FO.poisson_weights(7, 4, 200000))


def test_candidates_distinct_and_sized():
    c = FO.candidates(1, 2, 3, 62, FO.n_candidates("sqrt", 62))
    assert len(c) == 8 and len(set(c.tolist())) == 8 and c.max() < 62
    assert FO.n_candidates("all", 62) == 62 and FO.n_candidates("log2", 62) == 6
    assert FO.n_candidates("0.5", 62) == 31 and FO.n_candidates("onethird", 62) == 21


def test_hand_example_root_split():
    """Output j=0 equals feature 3; without bootstrap and with all features the root
    must split on feature 3 and the children are pure in output 0."""
    rng = np.random.default_rng(1)
    n = 400
    Xb = rng.integers(0, 2, size=(n, 62))
    Yb = np.zeros((n, 62), dtype=np.int64)
    Yb[:, 0] = Xb[:, 3]
    rf = RandomForest(n_trees=1, max_depth=1, feature_subset="all", bootstrap=False, device="cpu")
    rf.fit(FO.pack_bits(Xb), FO.pack_bits(Yb)[:, 0], 62)
    assert rf.feat[0, 0] == 3
    assert rf.value[0, 1, 0] == 0.0 and rf.value[0, 2, 0] == 1.0
    # gain = SL2/nL + SR2/nR - S2/n with S = per-output sums
    nR = int(Xb[:, 3].sum())
    expect = nR ** 2 / nR - nR ** 2 / n
    assert abs(rf.gain[0, 0] - expect) < 1e-9


def test_forest_learns_planted_and_is_deterministic(draws):
    ds, X, Y, F = draws
    ntr = 2000
    a = RandomForest(n_trees=12, max_depth=5, seed=9, device="cpu").fit(X[:ntr], Y[:ntr], F)
    b = RandomForest(n_trees=12, max_depth=5, seed=9, device="cpu").fit(X[:ntr], Y[:ntr], F)
    assert np.array_equal(a.feat, b.feat) and np.array_equal(a.value, b.value)
    p = a.predict_proba(X[ntr:])
    yt = multi_hot(ds.numbers[ntr + 1:])
    # structured prediction beats the all-zero floor on planted data
    top = np.argsort(-p[:, :50], 1)[:, :5]
    hits = np.take_along_axis(yt[:, :50], top, 1).sum(1).mean()
    assert hits > 5 * 5 / 50 * 1.5, hits


def test_save_load_roundtrip(tmp_path, draws):
    _, X, Y, F = draws
    rf = RandomForest(n_trees=3, max_depth=3, seed=1, device="cpu").fit(X[:500], Y[:500], F)
    p = tmp_path / "forest.npz"
    rf.save(str(p))
    back = RandomForest.load(str(p))
    assert np.array_equal(back.feat, rf.feat) and np.array_equal(back.value, rf.value)
    assert np.allclose(back.predict_proba(X[500:600]), rf.predict_proba(X[500:600]))


def test_tree_ids_make_shards_compose(draws):
    """Trees are keyed by global id: fitting [0,6) == fitting [0,3) + [3,6) (C5 tree-parallel)."""
    from euromillioner_amd.models.forest_oracle import grow_forest_numpy

    _, X, Y, F = draws
    full = grow_forest_numpy(X[:800], Y[:800], F, list(range(6)), 4, 8, 1, True, 5)
    a = grow_forest_numpy(X[:800], Y[:800], F, [0, 1, 2], 4, 8, 1, True, 5)
    b = grow_forest_numpy(X[:800], Y[:800], F, [3, 4, 5], 4, 8, 1, True, 5)
    for i in range(4):
        assert np.array_equal(full[i], np.concatenate([a[i], b[i]]))


@pytest.mark.gpu
# one feature word: record-form row lists (sqrt / log2 / all); two words (lags 2): index form.  Every
# histogram kernel must reproduce the oracle exactly
@pytest.mark.parametrize("depth,subset,boot,lags", [(5, "sqrt", True, 1), (3, "all", False, 1), (6, "0.3", True, 2),
                                                   (7, "log2", False, 1), (8, "sqrt", True, 1), (0, "sqrt", True, 1),
                                                   (1, "sqrt", True, 1), (2, "log2", False, 1)])
def test_hip_forest_matches_oracle(depth, subset, boot, lags):
    ds = DrawSet.synthetic(n=3000, seed=2, planted=0.7, calendar=False)
    X, Y, F = draw_features(ds.numbers, lags)
    gpu = RandomForest(n_trees=10, max_depth=depth, feature_subset=subset, bootstrap=boot, seed=11, device="cuda")
    gpu.fit(X, Y, F)
    assert gpu.backend_used == "hip"
    cpu = RandomForest(n_trees=10, max_depth=depth, feature_subset=subset, bootstrap=boot, seed=11, device="cpu")
    cpu.fit(X, Y, F)
    assert np.array_equal(gpu.feat, cpu.feat)
    live = gpu.feat > -2
    assert np.array_equal(gpu.value[live], cpu.value[live])
    assert np.array_equal(gpu.gain, cpu.gain)
    assert np.array_equal(gpu.cover[live], cpu.cover[live])
    pd = gpu.predict_proba_device(X[:700]).cpu().numpy()[:, :62]
    assert np.allclose(pd, cpu.predict_proba(X[:700]), atol=1e-6)


@pytest.mark.gpu
def test_hip_forest_predict_many_trees():
    """> 64 trees: the lane-parallel traversal runs in two passes (lanes = trees t0 .. t0+63)."""
    ds = DrawSet.synthetic(n=2000, seed=4, planted=0.7, calendar=False)
    X, Y, F = draw_features(ds.numbers, 1)
    gpu = RandomForest(n_trees=100, max_depth=4, seed=3, device="cuda")
    gpu.fit(X, Y, F)
    assert gpu.backend_used == "hip"
    pd = gpu.predict_proba_device(X[:500]).cpu().numpy()[:, :62]
    cpu = RandomForest(n_trees=100, max_depth=4, seed=3, device="cpu")
    cpu.fit(X, Y, F)
    assert np.array_equal(gpu.feat, cpu.feat)
    assert np.allclose(pd, cpu.predict_proba(X[:500]), atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [4, 8])
def test_hip_forest_predict_matches_torch_traversal(depth):
    """Deep trees on 20k rows: GPU predict == a plain torch traversal of the same device arrays."""
    import torch

    from euromillioner_amd.data.draws import mask_bits
    from euromillioner_amd.data.synthetic import generate_draws
    from euromillioner_amd.ops import forest as K

    nums, _ = generate_draws(20001, seed=0, planted=0.9, native=False)
    md = torch.from_numpy(mask_bits(nums).view(np.int64)).cuda()
    n_tr = 14000
    feat, value, _, _ = K.fit(md[:n_tr].reshape(-1, 1).contiguous(), md[1:n_tr + 1].contiguous(), 62, 0, 70, depth,
                              8, 1, True, 0, return_device=True)
    Xv = md[n_tr:20000].reshape(-1, 1).contiguous()
    p = K.predict(Xv, feat, value, depth)
    x = Xv[:, 0]
    acc = torch.zeros(Xv.shape[0], 64, device=x.device)
    for t in range(feat.shape[0]):
        nd = torch.zeros(Xv.shape[0], dtype=torch.long, device=x.device)
        for _ in range(depth + 1):
            f = feat[t][nd].long()
            nd = torch.where(f >= 0, 2 * nd + 1 + ((x >> f.clamp(min=0)) & 1), nd)
        acc += value[t][nd]
    ref = acc / feat.shape[0]
    assert torch.allclose(p[:, :62], ref[:, :62], atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("depth,trees,n", [(8, 100, 1), (8, 100, 777), (3, 37, 70001), (8, 100, 300001),
                                           (6, 129, 600000)])
def test_hip_forest_predict_streamed_bit_identical(depth, trees, n):
    """The tree-streamed predict (rf_predict_lds: LDS double-buffered trees, lane = row, rotated chunk
    order) equals the one-wave-per-row kernel bit for bit, for probabilities and logits, over row counts
    that give 1, 2 and 3 row groups per wave (and a grid past one workgroup per CU)."""
    import torch

    from euromillioner_amd.data.draws import mask_bits
    from euromillioner_amd.data.synthetic import generate_draws
    from euromillioner_amd.ops import forest as K

    nums, _ = generate_draws(20001, seed=1, planted=0.9, native=False)
    md = torch.from_numpy(mask_bits(nums).view(np.int64)).cuda()
    n_tr = 14000
    feat, value, _, _ = K.fit(md[:n_tr].reshape(-1, 1).contiguous(), md[1:n_tr + 1].contiguous(), 62, 0, trees, depth,
                              8, 1, True, 0, return_device=True)
    g = torch.Generator(device="cuda").manual_seed(n)
    Xv = md[torch.randint(0, 20000, (n,), device="cuda", generator=g)].reshape(-1, 1).contiguous()
    for logit in (False, True):
        a = K.predict(Xv, feat, value, depth, out_logit=logit)
        b = K.predict(Xv, feat, value, depth, out_logit=logit, stream_trees=False)
        assert torch.equal(a, b), (logit, float((a - b).abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("ymax", [7, 30])
def test_hip_forest_record_forms_match_oracle(ymax):
    """Rows with 0..7 outputs (absent positions included) take the position-form records, any row with
    more the mask form (rf_ycheck decides on the device): both equal the oracle."""
    rng = np.random.default_rng(ymax)
    n = 3000
    X = np.zeros(n, dtype=np.uint64)
    Y = np.zeros(n, dtype=np.uint64)
    for i in range(n):
        for b in rng.choice(62, size=int(rng.integers(0, 12)), replace=False):
            X[i] |= np.uint64(1) << np.uint64(b)
        for b in rng.choice(62, size=int(rng.integers(0, ymax)), replace=False):
            Y[i] |= np.uint64(1) << np.uint64(b)
        if i % 3 == 0:  # a learnable output
            Y[i] |= (X[i] & np.uint64(1)) << np.uint64(5)
    for depth, subset, boot in ((6, "sqrt", True), (4, "all", False)):
        g = RandomForest(n_trees=12, max_depth=depth, feature_subset=subset, bootstrap=boot, seed=7, device="cuda")
        g.fit(X.reshape(-1, 1), Y, 62)
        assert g.backend_used == "hip"
        c = RandomForest(n_trees=12, max_depth=depth, feature_subset=subset, bootstrap=boot, seed=7, device="cpu")
        c.fit(X.reshape(-1, 1), Y, 62)
        assert np.array_equal(g.feat, c.feat)
        live = g.feat > -2
        assert np.array_equal(g.value[live], c.value[live])
        assert np.array_equal(g.gain, c.gain)
        assert np.array_equal(g.cover[live], c.cover[live])
