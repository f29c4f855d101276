"""GPU numerics for the exact-fp32 MFMA GEMM (csrc/gemm_f32.hip) and the `--dtype fp32` trainer,
against plain PyTorch fp32 references (fp64 for the GEMM itself)."""
import pytest
import torch

from euromillioner_amd.data.draws import DrawSet, multi_hot

pytestmark = pytest.mark.gpu

ACT = {"none": lambda x: x, "relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh}
DACT = {"relu": lambda y: (y > 0).double(), "sigmoid": lambda y: y * (1 - y), "tanh": lambda y: 1 - y * y}


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize("M,N,K", [(300, 200, 70), (128, 128, 16), (1, 7, 5), (517, 1030, 333)])
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("act", ["none", "relu", "tanh"])
def test_gemm_f32_layouts_and_epilogue(M, N, K, a_kc, b_kc, act):
    from euromillioner_amd.ops import linear_f32 as LF

    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + 7 * K)
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(K, N, device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    a = A if a_kc else A.t().contiguous()
    b = B.t().contiguous() if b_kc else B
    out = torch.empty(M, N, device="cuda")
    LF.gemm_f32(a, a_kc, b, b_kc, out, M, N, K, bias=bias, act=act)
    ref = ACT[act](A.double() @ B.double() + bias.double())
    assert _rel(out, ref) < 1e-5  # exact fp32 products, fp32 accumulation


@pytest.mark.parametrize("dact", ["relu", "sigmoid", "tanh"])
def test_gemm_f32_dact_beta(dact):
    from euromillioner_amd.ops import linear_f32 as LF

    g = torch.Generator(device="cuda").manual_seed(5)
    M, N, K = 257, 130, 96
    A, B = torch.randn(M, K, device="cuda", generator=g), torch.randn(N, K, device="cuda", generator=g)
    Y = torch.sigmoid(torch.randn(M, N, device="cuda", generator=g)) if dact != "relu" else \
        torch.relu(torch.randn(M, N, device="cuda", generator=g))
    out = torch.empty(M, N, device="cuda")
    LF.gemm_f32(A, True, B, True, out, M, N, K, dact_src=Y, dact=dact)
    ref = (A.double() @ B.double().t()) * DACT[dact](Y.double())
    assert _rel(out, ref) < 1e-5
    C0 = torch.randn(M, N, device="cuda", generator=g)
    out2 = C0.clone()
    LF.gemm_f32(A, True, B, True, out2, M, N, K, alpha=0.5, beta=2.0)
    assert _rel(out2, 0.5 * (A.double() @ B.double().t()) + 2.0 * C0.double()) < 1e-5


def test_gemm_f32_split_k_wgrad():
    from euromillioner_amd.ops import linear_f32 as LF

    g = torch.Generator(device="cuda").manual_seed(9)
    Bn, Nn, K = 50000, 62, 64
    dz, x = torch.randn(Bn, Nn, device="cuda", generator=g), torch.randn(Bn, K, device="cuda", generator=g)
    out = torch.empty(Nn, K, device="cuda")
    LF.linear_wgrad(dz, x, out, parts_cache={})
    assert _rel(out, dz.double().t() @ x.double()) < 1e-5


def test_fp32_trainer_grads_match_torch():
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer
    from euromillioner_amd.models.mlp import DrawMLP
    from euromillioner_amd.ops.fused_mlp import rows_to_masks

    ds = DrawSet.synthetic(n=5000, seed=3, planted=0.6, calendar=False)
    masks = rows_to_masks(torch.from_numpy(ds.numbers).cuda())
    sizes, B, off = (62, 128, 62), 2048, 5
    tr = GemmMLPTrainer(sizes, seed=9, dtype="fp32")
    assert tr.shadow is None
    ref = DrawMLP(sizes, seed=9)
    X = torch.from_numpy(multi_hot(ds.numbers[off:off + B])).float()
    Y = torch.from_numpy(multi_hot(ds.numbers[off + 1:off + 1 + B])).float()
    l = ref.loss(ref(X), Y)
    l.backward()
    lk, gk = tr.grads_only(masks, B, offset=off)
    assert abs(lk - l.item()) < 1e-5 * max(1, l.item())
    for n, p in ref.named_parameters():
        assert _rel(gk[n].cpu(), p.grad) < 1e-4, n  # fp32 end to end: far tighter than the bf16 path


def test_fp32_cli_config_trains():
    from euromillioner_amd import config as C
    from euromillioner_amd.train import train

    cfg = C.build_config(None, {"model": "mlp", "device": "cuda", "mlp.dtype": "fp32", "data.n_draws": 6001,
                                "data.planted": 0.8, "mlp.steps": 80, "mlp.batch": 1024, "mlp.lr": 0.005,
                                "mlp.eval_every": 0, "log.level": "WARN"}, environ={})
    res = train(cfg)
    assert res["engine"] == "fused"  # 62->128->62 relu: the exact-fp32 fused kernel (csrc/mlp_fused_f32.hip)
    assert res["val"]["acc"] > res["val"]["trivial_acc"], res["val"]
    # any other stack takes the fp32 GEMM engine
    cfg = C.build_config(None, {"model": "mlp", "device": "cuda", "mlp.dtype": "fp32", "mlp.hidden": [96],
                                "data.n_draws": 6001, "data.planted": 0.8, "mlp.steps": 80, "mlp.batch": 1024,
                                "mlp.lr": 0.005, "mlp.eval_every": 0, "log.level": "WARN"}, environ={})
    res = train(cfg)
    assert res["engine"] == "gemm"
    assert res["val"]["acc"] > res["val"]["trivial_acc"], res["val"]
