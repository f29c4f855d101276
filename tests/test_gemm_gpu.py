"""GPU numerics for the MFMA GEMM (K1-K3), colsum, fused loss-grad (K10) and the GEMM-path
MLPs vs plain PyTorch fp32 references."""
import pytest
import torch

from euromillioner_amd.data.draws import DrawSet, multi_hot
from euromillioner_amd.models import losses as L

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.bfloat16().float()


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


ACT = {"none": lambda x: x, "relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh}
DACT = {"relu": lambda y: (y > 0).float(), "sigmoid": lambda y: y * (1 - y), "tanh": lambda y: 1 - y * y}


def _bf16_chain_grads(tr, X, Y, loss="softmax"):
    """fp32 reference of the GEMM trainer's step with the SAME bf16 roundings the kernels apply: bf16
    weights (the shadow), bf16 hidden activations and bf16 dL/dZ between layers; fp32 accumulation,
    fp32 weight / bias gradients.  What remains between it and the kernels is fp32 summation order, so
    a per-tensor tolerance of 1e-2 is tight: one zeroed bias column or weight row fails it."""
    sd = tr.state_dict()
    n_layers = len(tr.sizes) - 1
    Ws = [_bf(sd[f"layers.{i}.weight"].cuda().float()) for i in range(n_layers)]
    bs = [sd[f"layers.{i}.bias"].cuda().float() for i in range(n_layers)]
    hs = [X.cuda()]
    for i in range(n_layers - 1):
        hs.append(_bf(ACT[tr.activation](hs[-1] @ Ws[i].t() + bs[i])))
    logits = (hs[-1] @ Ws[-1].t() + bs[-1]).detach().requires_grad_()
    lv = L.LOSSES[loss](logits, Y.cuda())
    lv.backward()
    dz = _bf(logits.grad)
    out = {}
    for i in reversed(range(n_layers)):
        out[f"layers.{i}.weight"] = dz.t() @ hs[i]
        out[f"layers.{i}.bias"] = dz.sum(0)
        if i > 0:
            dz = _bf((dz @ Ws[i]) * DACT[tr.activation](hs[i]))
    return lv.item(), out


def _assert_tight(gk, ref, tol=1e-2):
    for n, g in ref.items():
        err = _rel(gk[n], g)
        assert err < tol, (n, err)


@pytest.mark.parametrize("M,N,K", [(300, 200, 70), (128, 128, 64), (1, 7, 5), (517, 1030, 333)])
@pytest.mark.parametrize("act", ["none", "relu", "sigmoid", "tanh"])
def test_forward_nt(M, N, K, act):
    from euromillioner_amd.ops import linear as LIN

    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
    b = torch.randn(N, device="cuda", generator=g)
    y = LIN.linear_fwd(LIN.aligned(x), LIN.aligned(w), b, act, torch.float32)
    ref = ACT[act](_bf(x) @ _bf(w).t() + b)
    assert y.shape == (M, N)
    assert _rel(y, ref) < 2e-3, _rel(y, ref)
    yb = LIN.linear_fwd(LIN.aligned(x), LIN.aligned(w), b, act, torch.bfloat16)
    assert _rel(yb, ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(300, 200, 70), (64, 8192, 64), (2048, 136, 1000), (512, 512, 768)])
@pytest.mark.parametrize("dact", ["none", "relu", "sigmoid", "tanh"])
def test_dgrad_nn(M, N, K, dact):  # (512, 512, 768): 256-tile shape, routed through w^T and the NT path
    from euromillioner_amd.ops import linear as LIN

    g = torch.Generator(device="cuda").manual_seed(3 + M + N)
    dz = torch.randn(M, N, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g)
    y = ACT["sigmoid" if dact == "sigmoid" else "tanh" if dact == "tanh" else "relu"](
        torch.randn(M, K, device="cuda", generator=g))
    yq = LIN.aligned(y)
    out = LIN.linear_dgrad(LIN.aligned(dz), LIN.aligned(w), yq, dact)
    ref = _bf(dz) @ _bf(w)
    yf = yq.float()
    if dact == "relu":
        ref = ref * (yf > 0)
    elif dact == "sigmoid":
        ref = ref * yf * (1 - yf)
    elif dact == "tanh":
        ref = ref * (1 - yf * yf)
    assert _rel(out, ref) < 1e-2, _rel(out, ref)


@pytest.mark.parametrize("M,N,K", [(1000, 62, 64), (4096, 200, 136), (77, 9, 13), (1024, 256, 512)])
def test_wgrad_tn_and_accumulate(M, N, K):  # (1024, 256, 512): alpha = 1 runs dz^T, x^T and the NT path
    from euromillioner_amd.ops import linear as LIN

    g = torch.Generator(device="cuda").manual_seed(M + K)
    dz = torch.randn(M, N, device="cuda", generator=g)
    x = torch.randn(M, K, device="cuda", generator=g)
    dzq, xq = LIN.aligned(dz), LIN.aligned(x)
    gw = LIN.linear_wgrad(dzq, xq)
    ref = _bf(dz).t() @ _bf(x)
    assert _rel(gw, ref) < 1e-4, _rel(gw, ref)
    gw2 = LIN.linear_wgrad(dzq, xq, out=gw.clone(), alpha=0.5, beta=1.0)
    assert _rel(gw2, 1.5 * ref) < 1e-4
    cs = LIN.colsum(dzq)
    assert _rel(cs, _bf(dz).sum(0)) < 1e-5


def test_large_square_gemm():
    from euromillioner_amd.ops import linear as LIN

    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn(4096, 4096, device="cuda", generator=g).bfloat16()
    b = torch.randn(4096, 4096, device="cuda", generator=g).bfloat16()
    y = LIN.linear_fwd(a, b, None, "none", torch.float32)
    ref = a.float() @ b.float().t()
    assert _rel(y, ref) < 1e-5


@pytest.fixture(scope="module")
def data():
    from euromillioner_amd.ops.fused_mlp import rows_to_masks

    ds = DrawSet.synthetic(n=5000, seed=3, planted=0.6, calendar=False)
    return ds, rows_to_masks(torch.from_numpy(ds.numbers).cuda())


@pytest.mark.parametrize("loss", ["softmax", "bce"])
def test_loss_grad_kernel(data, loss):
    from euromillioner_amd.ops import linear as LIN

    ds, masks = data
    B, off = 1001, 17
    g = torch.Generator(device="cuda").manual_seed(1)
    z = (3 * torch.randn(B, 64, device="cuda", generator=g)).requires_grad_()
    Y = torch.from_numpy(multi_hot(ds.numbers[off + 1:off + 1 + B])).cuda()
    ref = L.LOSSES[loss](z, Y)
    ref.backward()
    dz, part = LIN.loss_grad(z.detach(), masks, B, loss, offset=off, grad_scale=1.0 / B)
    assert abs(float(part.double().sum()) / B - ref.item()) < 1e-4 * max(1, ref.item())
    assert _rel(dz[:, :62], z.grad[:, :62]) < 1e-2
    assert float(dz[:, 62:].abs().max()) == 0.0


@pytest.mark.parametrize("act", ["relu", "tanh", "sigmoid"])
def test_drawmlp_hip_autograd_matches_fp32(data, act):
    from euromillioner_amd.models.mlp import DrawMLP

    ds, _ = data
    X = torch.from_numpy(multi_hot(ds.numbers[:700])).float()
    Y = torch.from_numpy(multi_hot(ds.numbers[1:701])).float()
    cpu = DrawMLP((62, 96, 40, 62), activation=act, seed=4)
    gpu = DrawMLP((62, 96, 40, 62), activation=act, seed=4).cuda()
    lc = cpu.loss(cpu(X), Y)
    lc.backward()
    lg = gpu.loss(gpu(X.cuda()), Y.cuda())
    lg.backward()
    assert abs(lc.item() - lg.item()) < 1e-2 * max(1, lc.item())
    for (n, pc), (_, pg) in zip(cpu.named_parameters(), gpu.named_parameters()):
        assert _rel(pg.grad.cpu(), pc.grad) < 5e-2, n


@pytest.mark.parametrize("sizes", [(62, 96, 40, 62), (62, 128, 62), (62, 300, 62)])
def test_gemm_trainer_grads_match_drawmlp(data, sizes):
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer
    from euromillioner_amd.models.mlp import DrawMLP

    ds, masks = data
    B, off = 2048, 5
    tr = GemmMLPTrainer(sizes, seed=9)
    ref = DrawMLP(sizes, seed=9)
    X = torch.from_numpy(multi_hot(ds.numbers[off:off + B])).float()
    Y = torch.from_numpy(multi_hot(ds.numbers[off + 1:off + 1 + B])).float()
    l = ref.loss(ref(X), Y)
    l.backward()
    lk, gk = tr.grads_only(masks, B, offset=off)
    assert abs(lk - l.item()) < 1e-2 * max(1, l.item())
    for n, p in ref.named_parameters():
        assert _rel(gk[n].cpu(), p.grad) < 5e-2, n
    _assert_tight(gk, _bf16_chain_grads(tr, X, Y)[1])
    # the pads of the flat buffers stay zero
    sd = tr.state_dict()
    for n, p in ref.named_parameters():
        assert torch.equal(sd[n], p.detach())


def test_gemm_trainer_learns_planted(data):
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer

    ds, masks = data
    tr = GemmMLPTrainer((62, 256, 256, 62), lr=3e-3, seed=0)
    ntr = 3800
    first = None
    for s in range(150):
        loss = tr.step(masks, ntr, offset=0)
        if first is None:
            first = loss.item()
    assert loss.item() < first
    ev = tr.evaluate(masks, 1000, offset=ntr)
    assert ev["acc"] > ev["trivial_acc"], ev


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 320), (1024, 256, 4096), (1024, 2048, 64),
                                   (768, 512, 128)])
@pytest.mark.parametrize("act", ["none", "relu", "sigmoid", "tanh"])
def test_big_nt_forward_with_transposed_copy(M, N, K, act):
    """K = 64 / 128 shapes run the skinny-K store-stream kernel (gemm_k64_kernel), the others the 256 tile."""
    from euromillioner_amd.ops import linear as LIN

    assert LIN.big_ok(M, N, K)
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    ct = torch.empty(N, M, dtype=torch.bfloat16, device="cuda")
    y = LIN.linear_fwd(x, w, b, act, torch.bfloat16, ct=ct)
    ref = ACT[act](x.float() @ w.float().t() + b)
    assert _rel(y, ref) < 1e-2, _rel(y, ref)
    assert torch.equal(ct, y.t())
    y32 = LIN.linear_fwd(x, w, None, "none", torch.float32)
    assert _rel(y32, x.float() @ w.float().t()) < 1e-5


@pytest.mark.parametrize("dact", ["relu", "sigmoid", "tanh"])
def test_big_nt_dgrad_and_wgrad(dact):
    from euromillioner_amd.ops import linear as LIN

    g = torch.Generator(device="cuda").manual_seed(7)
    M, N, K = 512, 256, 768
    dz = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    w = torch.randn(N, K, device="cuda", generator=g).bfloat16()
    y = ACT[dact](torch.randn(M, K, device="cuda", generator=g)).bfloat16()
    wt = LIN.transpose(w)
    assert torch.equal(wt, w.t())
    ct = torch.empty(K, M, dtype=torch.bfloat16, device="cuda")
    out = LIN.linear_dgrad_nt(dz, wt, y, dact, ct=ct)
    ref = dz.float() @ w.float()
    yf = y.float()
    ref = ref * ((yf > 0).float() if dact == "relu" else yf * (1 - yf) if dact == "sigmoid" else 1 - yf * yf)
    assert _rel(out, ref) < 1e-2, _rel(out, ref)
    assert torch.equal(ct, out.t())
    # wgrad through transposed copies: dW = dz^T @ x
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    gw = LIN.linear_wgrad_nt(LIN.transpose(dz), LIN.transpose(x))
    assert _rel(gw, dz.float().t() @ x.float()) < 1e-5
    assert _rel(LIN.rowsum(LIN.transpose(dz)), dz.float().sum(0)) < 1e-5


@pytest.mark.parametrize("dact,K", [("relu", 64), ("sigmoid", 128), ("relu", 768), ("tanh", 256)])
def test_dgrad_fused_bias_partials(dact, K):
    """The dgrad epilogue's column sums (fused bias gradient): colpart rows = sums over 128 output
    rows of the fp32 epilogue values; the fixed-order reduce equals dZ.sum(0) of the reference, and
    the bf16 output / transposed copy are unchanged by the extra work.  K = 64 / 128 exercise the
    skinny-K kernel (wave pairs combined through LDS), the others the 256-tile epilogue."""
    from euromillioner_amd.ops import linear as LIN

    g = torch.Generator(device="cuda").manual_seed(K)
    M, Kout = 1024, 512  # dz [M, K] (K = the reduction width) -> out [M, Kout]
    dz = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(dz.shape[1], Kout, device="cuda", generator=g) / dz.shape[1] ** 0.5).bfloat16()
    y = ACT[dact](torch.randn(M, Kout, device="cuda", generator=g)).bfloat16()
    wt = LIN.transpose(w)
    ct = torch.empty(Kout, M, dtype=torch.bfloat16, device="cuda")
    part = torch.full(((M // 128) * Kout,), float("nan"), device="cuda")
    out = LIN.linear_dgrad_nt(dz, wt, y, dact, ct=ct, colpart=part)
    yf = y.float()
    ref = (dz.float() @ w.float()) * ((yf > 0).float() if dact == "relu" else yf * (1 - yf) if dact == "sigmoid"
                                       else 1 - yf * yf)
    assert _rel(out, ref) < 1e-2, _rel(out, ref)
    assert torch.equal(ct, out.t())
    assert torch.isfinite(part).all()  # every partial row written
    db = torch.empty(Kout, device="cuda")
    LIN.colpart_reduce(part, M // 128, Kout, db)
    assert _rel(db, ref.sum(0)) < 1e-4, _rel(db, ref.sum(0))
    blocks = ref.view(M // 128, 128, Kout).sum(1)
    assert _rel(part.view(M // 128, Kout), blocks) < 1e-4
    db2 = db.clone()
    LIN.colpart_reduce(part, M // 128, Kout, db2, accumulate=True)
    assert torch.allclose(db2, 2 * db, rtol=1e-6, atol=1e-6)


def _pack_bits(y: torch.Tensor) -> torch.Tensor:
    """(y > 0) packed as the kernels' activity bits: int32 [M / 32, N], bit k of word [r, n] = y[32r + k, n] > 0."""
    M, N = y.shape
    pos = (y.float() > 0).long().view(M // 32, 32, N)
    words = (pos << torch.arange(32, device=y.device).view(1, 32, 1)).sum(1)
    return torch.where(words >= 2 ** 31, words - 2 ** 32, words).to(torch.int32)


@pytest.mark.parametrize("M,N,K", [(256, 512, 64), (512, 768, 320), (1024, 256, 128)])
def test_relu_bits_forward_and_dgrad(M, N, K):
    """ReLU activity bits: the forward epilogue writes (y > 0) packed 32 rows per word next to an unchanged
    bf16 output (K = 64 / 128: skinny-K kernel, else the 256 tile), and a relu dgrad reading the bits is
    bit-identical (output, C^T, bias partials) to the one reading the bf16 activation, on both the skinny-K
    (reduction 64) and the 256-tile (reduction 256) dgrad."""
    from euromillioner_amd.ops import linear as LIN

    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    bits = LIN.relu_bits(M, N, "cuda").fill_(0x5A5A5A5A)
    y = LIN.linear_fwd(x, w, b, "relu", torch.bfloat16, bits=bits)
    assert torch.equal(y, LIN.linear_fwd(x, w, b, "relu", torch.bfloat16))
    assert torch.equal(bits, _pack_bits(y))
    assert 0.3 < (y > 0).float().mean().item() < 0.7
    for R in (64, 256):
        dz = torch.randn(M, R, device="cuda", generator=g).bfloat16()
        wt = LIN.transpose((torch.randn(R, N, device="cuda", generator=g) / R ** 0.5).bfloat16())
        outs = []
        for use_bits in (False, True):
            ct = torch.empty(N, M, dtype=torch.bfloat16, device="cuda")
            part = torch.full(((M // 128) * N,), float("nan"), device="cuda")
            o = LIN.linear_dgrad_nt(dz, wt, y, "relu", ct=ct, colpart=part, bits=bits if use_bits else None)
            outs.append((o, ct, part))
        for a, c in zip(*outs):
            assert torch.equal(a, c)
    with pytest.raises(ValueError):
        LIN.linear_fwd(x, w, b, "tanh", torch.bfloat16, bits=bits)


@pytest.mark.parametrize("M,N", [(256, 256), (768, 512)])
def test_big_mn_operands_exact_and_repeatable(M, N):
    """The 256-tile kernel reading MN-contiguous operands in place (csrc/gemm.hip GPanel, g_frag): the wgrad
    layout (both operands [K][rows]) and the dgrad layout (B [K][cols]) at 1..40 K-tiles, on exact
    asymmetric small-integer operands (every fp32 sum exact, so a mis-swizzled or transposed LDS read of
    either operand cannot cancel out), and bitwise repeatable over 4 launches."""
    from euromillioner_amd.ops import linear as LIN

    for K in (64, 128, 320, 2560):
        kk = torch.arange(K, device="cuda").view(K, 1)
        a = ((3 * kk + 5 * torch.arange(M, device="cuda").view(1, M)) % 7 - 3).bfloat16()   # [K, M]
        b = ((2 * kk + 7 * torch.arange(N, device="cuda").view(1, N)) % 11 - 5).bfloat16()  # [K, N]
        ref = a.double().t() @ b.double()
        out = torch.full((M, N), float("nan"), device="cuda")
        LIN.gemm(a, False, b, False, out, M, N, K)
        assert torch.equal(out.double(), ref), (M, N, K)
        for _ in range(3):
            again = LIN.gemm(a, False, b, False, torch.empty_like(out), M, N, K)
            assert torch.equal(again, out)
        # dgrad layout: A [M][K] K-contiguous, B [K][N] MN-contiguous, bf16 out (one rounding of an exact sum)
        at = a.t().contiguous()
        outb = LIN.gemm(at, True, b, False, torch.empty(M, N, dtype=torch.bfloat16, device="cuda"), M, N, K)
        assert torch.equal(outb, ref.float().bfloat16()), (M, N, K)


@pytest.mark.parametrize("dact", ["relu", "tanh"])
def test_big_mn_forms_bitwise_equal_nt(dact):
    """The MN-operand forms of the 256-tile kernel (``gemm(..., a_kc / b_kc = False)``: dgrad reading w in
    place, wgrad reading dz and x in place) are bitwise the NT kernel on explicitly transposed copies -- same
    MFMA order, same epilogue: output, bias partials, relu-bits act'; a column-panel view of dz (the DP wgrad
    panels) gives the matching rows of the whole wgrad, and beta = 1 accumulates exactly."""
    from euromillioner_amd.ops import linear as LIN

    g = torch.Generator(device="cuda").manual_seed(11)
    M, N, K = 1024, 512, 768
    dz = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / N ** 0.5).bfloat16()
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = torch.randn(K, device="cuda", generator=g) * 0.1
    bits = LIN.relu_bits(M, K, "cuda") if dact == "relu" else None
    xw = (torch.randn(K, 256, device="cuda", generator=g) / 16).bfloat16()
    y = LIN.linear_fwd(LIN.aligned(torch.randn(M, 256, device="cuda", generator=g).bfloat16()), xw, b, dact,
                       torch.bfloat16, bits=bits)
    res = []
    for wm, kc in ((w, False), (LIN.transpose(w), True)):
        part = torch.full(((M // 128) * K,), float("nan"), device="cuda")
        o = torch.empty(M, K, dtype=torch.bfloat16, device="cuda")
        LIN.gemm(dz, True, wm, kc, o, M, K, N, dact_src=None if bits is not None else y, dact=dact, colpart=part,
                 bits=bits)
        res.append((o, part))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    gw = LIN.gemm(dz, False, x, False, torch.empty(N, K, device="cuda"), N, K, M)
    assert torch.equal(gw, LIN.linear_wgrad_nt(LIN.transpose(dz), LIN.transpose(x)))
    panel = LIN.gemm(dz[:, 256:512], False, x, False, torch.empty(256, K, device="cuda"), 256, K, M)
    assert torch.equal(panel, gw[256:512])
    acc = LIN.gemm(dz, False, x, False, gw.clone(), N, K, M, beta=1.0)
    assert torch.equal(acc, gw + gw)


def test_wgrad_split_k_and_colsum_big_batch():
    from euromillioner_amd.ops import linear as LIN

    g = torch.Generator(device="cuda").manual_seed(8)
    M = 65536
    dz = torch.randn(M, 64, device="cuda", generator=g).bfloat16()
    x = torch.randn(M, 200, device="cuda", generator=g).bfloat16()
    xq = LIN.aligned(x)
    gw = LIN.linear_wgrad(dz, xq)
    ref = dz.double().t() @ x.double()
    assert _rel(gw.double(), ref) < 1e-5
    assert _rel(LIN.colsum(dz).double(), dz.double().sum(0)) < 1e-5


def test_gemm_trainer_big_plan_matches_drawmlp(data):
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer
    from euromillioner_amd.models.mlp import DrawMLP

    ds, masks = data
    sizes, B, off = (62, 512, 256, 62), 1024, 3
    tr = GemmMLPTrainer(sizes, seed=2)
    plan = tr._plan(B)
    assert plan["wgrad"][1] and plan["dgrad"][1] and plan["dgrad"][2]
    ref = DrawMLP(sizes, seed=2)
    X = torch.from_numpy(multi_hot(ds.numbers[off:off + B])).float()
    Y = torch.from_numpy(multi_hot(ds.numbers[off + 1:off + 1 + B])).float()
    l = ref.loss(ref(X), Y)
    l.backward()
    lk, gk = tr.grads_only(masks, B, offset=off)
    assert abs(lk - l.item()) < 1e-2 * max(1, l.item())
    for n, p in ref.named_parameters():
        assert _rel(gk[n].cpu(), p.grad) < 5e-2, n
    # the bias gradients of layers 0 and 1 come from the 256-tile dgrad epilogues (fused colsum partials)
    _assert_tight(gk, _bf16_chain_grads(tr, X, Y)[1])


def test_fused_bias_partials_catch_a_dropped_column(data):
    """The tight reference rejects a bias gradient with ONE column zeroed (the check the fused
    bias-gradient epilogue is held to): mutation test of _assert_tight itself."""
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer

    ds, masks = data
    sizes, B, off = (62, 512, 256, 62), 1024, 3
    tr = GemmMLPTrainer(sizes, seed=2)
    X = torch.from_numpy(multi_hot(ds.numbers[off:off + B])).float()
    Y = torch.from_numpy(multi_hot(ds.numbers[off + 1:off + 1 + B])).float()
    _, gk = tr.grads_only(masks, B, offset=off)
    ref = _bf16_chain_grads(tr, X, Y)[1]
    _assert_tight(gk, ref)
    for name in ("layers.0.bias", "layers.1.bias", "layers.2.bias"):
        bad = dict(gk)
        bad[name] = gk[name].clone()
        bad[name][int(gk[name].abs().argmax())] = 0.0
        with pytest.raises(AssertionError):
            _assert_tight(bad, ref)


@pytest.mark.parametrize("M,N,K,big", [(256, 512, 256, True), (128, 96, 128, False), (300, 200, 300, False)])
def test_identity_a_asymmetric_b(M, N, K, big):
    """A = I with an asymmetric B catches a transposed C write (cdna_hip_programming.md 3)."""
    from euromillioner_amd.ops import linear as LIN

    assert LIN.big_ok(M, N, K) == big
    n = min(M, K)
    a = torch.zeros(M, K, device="cuda")
    a[torch.arange(n), torch.arange(n)] = 1.0
    # exact small integers, asymmetric: B[n][k] = (3n + 7k) % 17 - 8
    nn_, kk = torch.meshgrid(torch.arange(N, device="cuda"), torch.arange(K, device="cuda"), indexing="ij")
    w = ((3 * nn_ + 7 * kk) % 17 - 8).float()
    y = LIN.linear_fwd(LIN.aligned(a), LIN.aligned(w), None, "none", torch.float32)
    ref = a @ w.t()
    assert torch.equal(y, ref)


@pytest.mark.parametrize("M,N", [(256, 256), (768, 512), (2048, 1024)])
def test_big_nt_schedule_race_screen(M, N):
    """The 256x256 ping-pong K loop (gemm.hip gemm256_pp_kernel) at 1..40 K-tiles: every tail of its
    staging schedule, fp32 output vs the fp32 product of the same bf16 operands, and bitwise
    repeatable over 8 launches (a mis-ordered LDS-DMA read shows up as a non-repeatable tile)."""
    from euromillioner_amd.ops import linear as LIN

    for K in (64, 128, 192, 320, 2560):
        assert LIN.big_ok(M, N, K)
        g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
        x = torch.rand(M, K, device="cuda", generator=g).mul(2).sub(1).bfloat16()
        w = torch.rand(N, K, device="cuda", generator=g).mul(2).sub(1).bfloat16()
        ref = x.double() @ w.double().t()
        first = LIN.linear_fwd(x, w, None, "none", torch.float32)
        assert float((first.double() - ref).abs().max()) < 1e-4 * K ** 0.5, (M, N, K)
        for _ in range(7):
            again = LIN.linear_fwd(x, w, None, "none", torch.float32)
            assert torch.equal(again, first), (M, N, K)


@pytest.mark.parametrize("M,J,W,wide_dz", [(8192, 64, 512, False), (8192, 62, 768, False), (4096, 64, 256, True),
                                           (12288, 62, 512, True)])
def test_wgrad_skinny_matches_fp32(M, J, W, wide_dz):
    """The streaming skinny wgrad (64 x W over a big batch; both orientations, 62-wide padded
    operands, alpha/beta accumulate) vs the fp32 product of the same bf16 operands."""
    from euromillioner_amd.ops import linear as LIN

    g = torch.Generator(device="cuda").manual_seed(M + J + W)
    narrow = LIN.aligned(torch.randn(M, J, device="cuda", generator=g))
    wide = LIN.aligned(torch.randn(M, W, device="cuda", generator=g))
    dz, x = (wide, narrow) if wide_dz else (narrow, wide)
    assert LIN._skinny_ok(dz, x, LIN.empty_aligned(dz.shape[1], x.shape[1], torch.float32, dz.device))
    gw = LIN.linear_wgrad(dz, x)
    ref = dz.double().t() @ x.double()
    assert gw.shape == ref.shape
    assert _rel(gw.double(), ref) < 1e-5, _rel(gw.double(), ref)
    gw2 = LIN.linear_wgrad(dz, x, out=gw.clone(), alpha=0.5, beta=1.0)
    assert _rel(gw2.double(), 1.5 * ref) < 1e-5
    again = LIN.linear_wgrad(dz, x)
    assert torch.equal(again, gw)  # fixed-order slice reduction: bitwise repeatable


def test_gemm_trainer_odd_wide_layers_take_the_tile_path(data):
    """Hidden 1000 pads to 1024 (relu, bf16): the 256-tile GEMMs run every layer, the pad units stay
    exactly zero through a step, and the gradients still match the fp32 DrawMLP."""
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer
    from euromillioner_amd.models.mlp import DrawMLP

    ds, masks = data
    sizes, B, off = (62, 1000, 1000, 62), 1024, 7
    tr = GemmMLPTrainer(sizes, seed=4, lr=1e-3)
    assert tr.padded == (64, 1024, 1024, 64)
    plan = tr._plan(B)
    assert plan["wgrad"][1] and plan["dgrad"][1] and plan["dgrad"][2]
    ref = DrawMLP(sizes, seed=4)
    X = torch.from_numpy(multi_hot(ds.numbers[off:off + B])).float()
    Y = torch.from_numpy(multi_hot(ds.numbers[off + 1:off + 1 + B])).float()
    l = ref.loss(ref(X), Y)
    l.backward()
    lk, gk = tr.grads_only(masks, B, offset=off)
    assert abs(lk - l.item()) < 1e-2 * max(1, l.item())
    for n, p in ref.named_parameters():
        assert _rel(gk[n].cpu(), p.grad) < 5e-2, n
    _assert_tight(gk, _bf16_chain_grads(tr, X, Y)[1])
    tr.step(masks, B, offset=off)
    torch.cuda.synchronize()
    w1, _ = tr._views(tr.params, 1)  # [1024, 1024]: rows/cols 1000.. are padding
    assert float(w1[1000:].abs().max()) == 0.0 and float(w1[:, 1000:].abs().max()) == 0.0
