"""Property test of the raw GEMM entry point (ops/linear.gemm -> em_gemm_bf16) over random shapes,
both operand layouts, fp32/bf16 outputs, fused activations, act' masks and beta accumulation,
against a plain PyTorch fp32 reference of the same bf16 operands.  Shapes straddle the 256-tile
path (M, N multiples of 256, K of 64) and the any-layout 128-tile path, including 1-wide edges."""
import pytest
import torch
from hypothesis import HealthCheck, example, given, settings
from hypothesis import strategies as st

pytestmark = pytest.mark.gpu

ACT = {"none": lambda x: x, "relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh}
DACT = {"relu": lambda y: (y > 0).float(), "sigmoid": lambda y: y * (1 - y), "tanh": lambda y: 1 - y * y}


@st.composite
def cases(draw):
    big = draw(st.booleans())
    M = draw(st.sampled_from([256, 512]) if big else st.integers(1, 300))
    N = draw(st.sampled_from([256, 512]) if big else st.integers(1, 300))
    K = draw(st.sampled_from([64, 192, 640]) if big else st.integers(1, 300))
    a_kc, b_kc = draw(st.booleans()), draw(st.booleans())
    if big:
        a_kc = b_kc = draw(st.booleans()) or (a_kc and b_kc)
    out_bf16 = draw(st.booleans())
    mode = draw(st.sampled_from(["plain", "act", "dact", "beta"] if not out_bf16 else ["plain", "act", "dact"]))
    if mode == "beta":
        out_bf16 = False
    act = draw(st.sampled_from(["relu", "sigmoid", "tanh"]))
    seed = draw(st.integers(0, 2 ** 16))
    return M, N, K, a_kc, b_kc, out_bf16, mode, act, seed


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(cases())
# 256-tile shapes with an fp32 output and a fused act / act' (the 256 path has no fp32 act epilogue:
# these must fall back to the any-layout kernel, not fail)
@example((256, 512, 192, True, True, False, "act", "relu", 1))
@example((512, 256, 64, True, True, False, "dact", "tanh", 2))
@example((256, 256, 640, False, False, True, "dact", "sigmoid", 3))
def test_gemm_matches_fp32_reference(case):
    from euromillioner_amd.ops import linear as LIN

    M, N, K, a_kc, b_kc, out_bf16, mode, act, seed = case
    g = torch.Generator(device="cuda").manual_seed(seed)
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    B = (torch.randn(N, K, device="cuda", generator=g) / max(1, K) ** 0.5).bfloat16()
    a = LIN.aligned(A if a_kc else A.t().contiguous())
    b = LIN.aligned(B if b_kc else B.t().contiguous())
    ref = A.float() @ B.float().t()
    out = LIN.empty_aligned(M, N, torch.bfloat16 if out_bf16 else torch.float32, "cuda")
    kw = {}
    if mode == "act":
        bias = torch.randn(N, device="cuda", generator=g)
        kw = dict(bias=bias, act=act)
        ref = ACT[act](ref + bias)
    elif mode == "dact":
        y = LIN.aligned(ACT[act](torch.randn(M, N, device="cuda", generator=g)).bfloat16())
        kw = dict(dact_src=y, dact=act)
        ref = ref * DACT[act](y.float())
    elif mode == "beta":
        out.copy_(torch.randn(M, N, device="cuda", generator=g))
        kw = dict(beta=0.5, alpha=2.0)
        ref = 2.0 * ref + 0.5 * out.clone()
    LIN.gemm(a, a_kc, b, b_kc, out, M, N, K, **kw)
    err = float((out.float() - ref).abs().max())
    scale = float(ref.abs().max().clamp_min(1.0))
    tol = 2e-2 if out_bf16 else 2e-3
    assert err <= tol * scale, (case, err, scale)
