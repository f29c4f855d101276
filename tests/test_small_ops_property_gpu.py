"""Property tests of the small HIP ops over random shapes against plain PyTorch: bf16 transpose,
fp32 column / row sums of bf16 matrices (with accumulate and scale), the fp32 -> bf16 cast, the
flat Adam (fp32 and bf16 gradients, several steps, weight decay, odd lengths) and the one-hot lag
window encoder."""
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

pytestmark = pytest.mark.gpu
SET = settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@SET
@given(st.integers(1, 700), st.integers(1, 700), st.integers(0, 99))
def test_transpose_random(R, Cc, seed):
    from euromillioner_amd.ops import linear as LIN

    g = torch.Generator(device="cuda").manual_seed(seed)
    x = LIN.aligned(torch.randn(R, Cc, device="cuda", generator=g).bfloat16())
    assert torch.equal(LIN.transpose(x), x.t())


@SET
@given(st.integers(1, 3000), st.integers(1, 300), st.booleans(), st.sampled_from([1.0, 0.25]), st.integers(0, 99))
def test_colsum_rowsum_random(M, N, acc, scale, seed):
    from euromillioner_amd.ops import linear as LIN

    g = torch.Generator(device="cuda").manual_seed(seed)
    x = LIN.aligned(torch.randn(M, N, device="cuda", generator=g).bfloat16())
    base_c = torch.randn(N, device="cuda", generator=g)
    base_r = torch.randn(M, device="cuda", generator=g)
    c = LIN.colsum(x, out=base_c.clone(), accumulate=acc, scale=scale)
    r = LIN.rowsum(x, out=base_r.clone(), accumulate=acc, scale=scale)
    xf = x.double()
    ref_c = scale * xf.sum(0) + (base_c.double() if acc else 0)
    ref_r = scale * xf.sum(1) + (base_r.double() if acc else 0)
    assert torch.allclose(c.double(), ref_c, atol=1e-3, rtol=1e-4)
    assert torch.allclose(r.double(), ref_r, atol=1e-3, rtol=1e-4)


@SET
@given(st.integers(1, 100000), st.integers(0, 99))
def test_cast_bf16_random(n, seed):
    from euromillioner_amd.ops import fused_mlp as FM

    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(n, device="cuda", generator=g) * 100
    out = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    FM.cast_bf16(x, out)
    assert torch.equal(out, x.bfloat16())


@settings(max_examples=12, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.integers(1, 50000), st.booleans(), st.sampled_from([0.0, 0.01]), st.integers(0, 99))
def test_adam_flat_random(n, bf16_grad, wd, seed):
    from euromillioner_amd.ops import fused_mlp as FM

    g = torch.Generator(device="cuda").manual_seed(seed)
    p = torch.randn(n, device="cuda", generator=g)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    hp = torch.tensor([1e-3, 0.9, 0.999, 1e-8, wd], device="cuda")
    state = torch.zeros(2, dtype=torch.int32, device="cuda")
    ref = p.clone().requires_grad_()
    opt = torch.optim.Adam([ref], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd)  # L2 (g + wd w)
    for _ in range(3):
        gr = torch.randn(n, device="cuda", generator=g)
        if bf16_grad:
            gr = gr.bfloat16()
        FM.adam_flat(p, gr, m, v, hp, state)
        ref.grad = gr.float().clone()
        opt.step()
    torch.cuda.synchronize()
    assert torch.allclose(p, ref.detach(), atol=1e-6, rtol=1e-5), float((p - ref).abs().max())


@SET
@given(st.integers(1, 5000), st.integers(1, 4), st.integers(0, 50), st.booleans())
def test_onehot_lags_random(B, lags, offset, fp32):
    from euromillioner_amd.data.draws import DrawSet, multi_hot
    from euromillioner_amd.ops import fused_mlp as FM
    from euromillioner_amd.ops.fused_mlp import rows_to_masks

    ds = DrawSet.synthetic(n=B + lags + offset + 2, seed=B, planted=0.5, calendar=False)
    draws = rows_to_masks(torch.from_numpy(ds.numbers).cuda())
    out = FM.onehot_lags(draws, B, lags, offset=offset, dtype=torch.float32 if fp32 else torch.bfloat16)
    mh = torch.from_numpy(multi_hot(ds.numbers)).cuda().float()
    ref = torch.zeros(B, 64 * lags, device="cuda")
    for k in range(lags):
        ref[:, 64 * k:64 * k + 62] = mh[offset + k:offset + k + B]
    assert torch.equal(out.float(), ref)


def test_adam_bias_correction_exact_first_steps():
    """From zero weights every Adam update is visible at full fp32 precision, so the first steps'
    bias corrections (1 - beta^t, computed in fp64) must match torch.optim.Adam to ~fp32 rounding:
    a native exp/log form of beta^t (~1e-4 relative error at small t) fails this by 10x."""
    from euromillioner_amd.ops import fused_mlp as FM

    n = 4096
    g = torch.Generator(device="cuda").manual_seed(7)
    p = torch.zeros(n, device="cuda")
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    hp = torch.tensor([1e-2, 0.9, 0.999, 1e-8, 0.0], device="cuda")
    state = torch.zeros(2, dtype=torch.int32, device="cuda")
    ref = p.clone().requires_grad_()
    opt = torch.optim.Adam([ref], lr=1e-2, betas=(0.9, 0.999), eps=1e-8)
    for _ in range(6):
        gr = torch.randn(n, device="cuda", generator=g)
        FM.adam_flat(p, gr, m, v, hp, state)
        ref.grad = gr.clone()
        opt.step()
        torch.cuda.synchronize()
        assert torch.allclose(p, ref.detach(), rtol=5e-6, atol=5e-8), float((p - ref.detach()).abs().max())
