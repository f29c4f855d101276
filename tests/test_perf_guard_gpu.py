"""Performance guards for the two hot paths, loose enough for box-to-box variance and tight enough to
catch a structural regression (e.g. the run-time staging-lead flag in the GEMM's K loop that cost
~15 %, profiles/gemm_box_variance.md).

* 256-tile GEMM: our kernel against hipBLASLt (torch.matmul) on the same GPU, same call.  Measured
  ratio 0.88-0.90 on 8192^3; the regressed build ran at 0.78.
* fused 62->128->62 train step at 1M samples (train kernel + Adam, 10-step hipGraph): 80-84 us on the
  round-6 boxes (88-92 before the round-6 K7 work); the guard is 100 us.
"""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.perf]


def _time(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def test_gemm_256_tile_within_reach_of_hipblaslt():
    from euromillioner_amd.ops import linear as LIN

    H = 8192
    g = torch.Generator(device="cuda").manual_seed(0)
    x = (torch.rand(H, H, device="cuda", generator=g) - 0.5).bfloat16()
    w = (torch.rand(H, H, device="cuda", generator=g) - 0.5).bfloat16()
    y = torch.empty(H, H, device="cuda", dtype=torch.bfloat16)
    best = 0.0
    for _ in range(2):  # the better of two rounds: one clock hiccup must not fail the guard
        t_ours = _time(lambda: LIN.linear_fwd(x, w, None, "none", out=y), 10)
        t_lib = _time(lambda: torch.nn.functional.linear(x, w), 10)
        best = max(best, t_lib / t_ours)
    # 0.82: catches the regressed build (0.78) with ~7 % of the measured 0.88-0.90 to spare for the ratio's
    # box-to-box spread (both sides run on the same box, in the same process: the ratio moves far less than the
    # absolute times, profiles/gemm_box_variance.md); EUROM_PERF_GEMM_FLOOR overrides it
    import os

    floor = float(os.environ.get("EUROM_PERF_GEMM_FLOOR", "0.82"))
    assert best > floor, f"256-tile GEMM at {best:.2f} x hipBLASLt throughput (measured 0.88-0.90)"


def test_fused_step_time():
    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.mlp import FusedSmallMLP

    B = 1 << 20
    draws = generate_masks(B + 4096, seed=1, planted=0.9)
    m = FusedSmallMLP("cuda", lr=1e-3)
    m.step(draws, B, offset=0)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(gr, stream=s):
            for _ in range(10):
                m.step(draws, B, offset=0)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(200):  # past the clock ramp (~100 ms of load)
        gr.replay()
    torch.cuda.synchronize()
    us = min(_time(gr.replay, 20) for _ in range(2)) * 1e3 / 10
    assert us < 100.0, f"fused 1M-sample step {us:.1f} us (measured 80-84 us)"
