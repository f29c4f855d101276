"""The xGMI exchange protocol at world 4 and 8 in ONE process on one GPU.

Ranks sharing a device cannot co-schedule safely beyond two processes (parallel/xgmi.py
MAX_RANKS_PER_DEVICE), so the multi-process test covers world 2 only on the pool's 1-GPU boxes.  Here
rank 0 is real and its N - 1 peers are buffers of this process (``em_xgmi_connect_local``), played by
emulator kernels that copy rank 0's published data into the peers' slots and raise their flags, as the
peers' own consumers would:

* the generic stage / reduce collective over 8 consecutive steps (both slots four times): bit-exact
  rank-order sums of a vector that changes every step (a slot-parity or reuse error reads the data of
  two steps before);
* the fused DP optimizer step (train kernel -> ``em_adam_slab_xgmi``, block flags) over 8 steps against
  the same model stepped through the host path (slab reduce, a torch rank-order sum, Adam from the
  summed gradient): parameters and loss bit-identical at every step, with one block per slice and with
  the capped grid of ranks that share a device (blocks looping over slices);
* a peer that never publishes: the consumer's bounded wait expires and the error word is raised.

Reference parity: the C1 gradient all-reduce of BASELINE.json configs[2] (the reference itself has no
collectives).
"""
import ctypes

import pytest

pytestmark = pytest.mark.gpu


def _comms(world, n, timeout_s):
    from euromillioner_amd.ops import _native as N
    from euromillioner_amd.parallel import xgmi as XG  # noqa: F401  (signatures)

    hs = []
    for _ in range(world):
        h = ctypes.c_void_p()
        assert N.lib().em_xgmi_create(n, float(timeout_s), ctypes.byref(h)) == 0
        hs.append(h)
    arr = (ctypes.c_void_p * world)(*[h.value for h in hs])
    N.call("em_xgmi_connect_local", hs[0], world, 0, arr)
    return hs


def _error(h) -> int:
    from euromillioner_amd.ops import _native as N

    e = ctypes.c_int(0)
    N.call("em_xgmi_error", h, ctypes.byref(e))
    return int(e.value)


def _destroy(hs):
    from euromillioner_amd.ops import _native as N

    for h in hs:
        N.lib().em_xgmi_destroy(h)


@pytest.mark.parametrize("world", [4, 8])
def test_proxy_generic_allreduce_reuses_slots(world):
    import torch

    from euromillioner_amd.ops import _native as N

    dev = torch.device("cuda", 0)
    n = 4099
    hs = _comms(world, n, 10.0)
    try:
        idx = torch.arange(n, device=dev, dtype=torch.float32)
        stream = N.stream_handle(dev)
        for step in range(8):
            x = (step + 1) * 3.0 + idx * 0.25 - (step % 3) * 1024.0
            N.call("em_xgmi_stage", hs[0], x.data_ptr(), n, stream)
            N.call("em_xgmi_emulate_peers", hs[0], n, 0.0, stream)  # peers publish copies of x
            out = torch.empty_like(x)
            N.call("em_xgmi_reduce", hs[0], out.data_ptr(), n, 1.0, stream)
            want = x.clone()
            for _ in range(1, world):
                want = want + x
            torch.cuda.synchronize()
            assert _error(hs[0]) == 0, step
            assert torch.equal(out, want), (step, float((out - want).abs().max()))
    finally:
        torch.cuda.synchronize()
        _destroy(hs)


@pytest.mark.parametrize("world,max_blocks", [(4, 0), (8, 0), (8, 64)])
def test_proxy_fused_dp_step_bit_identical(world, max_blocks):
    import torch

    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.ops import _native as N
    from euromillioner_amd.ops import fused_mlp as FM

    dev = torch.device("cuda", 0)
    P = FM.P_TOTAL
    B = 65536
    draws = generate_masks(4 * B + 16, seed=3, planted=0.8, device=dev)
    a = FusedSmallMLP(dev, lr=2e-3, seed=1)  # proxy rank 0 of `world`
    r = FusedSmallMLP(dev, lr=2e-3, seed=1)  # host-path reference
    hs = _comms(world, P + 1, 10.0)
    side = torch.cuda.Stream(dev)
    scale = 1.0 / (B * world)
    try:
        for step in range(8):
            off = (step % 4) * B
            # proxy: the two-launch DP step, peers emulated beside the consumer on a side stream
            nslab = a._partials(draws, B, off, None, check=step == 0, step=a.state)
            ev = torch.cuda.Event()
            ev.record()
            side.wait_event(ev)
            with torch.cuda.stream(side):
                N.call("em_xgmi_emulate_block_peers", hs[0], P // 64, P + 1, 1, 0.0, N.stream_handle(dev))
            FM.adam_slab_xgmi(hs[0].value, a.slabs, nslab, scale, a.params, a.m, a.v, a.hp, a.state, a.loss_slabs,
                              img=a.img, loss_out=a.loss_out, loss_scale=scale, pre=True, max_blocks=max_blocks)
            torch.cuda.current_stream().wait_stream(side)
            # reference: this rank's reduced [grad | loss], summed over `world` equal ranks in rank order
            nslab = r._partials(draws, B, off, None, check=step == 0, step=r.state)
            FM.adam_slab(r.slabs, nslab, scale, r.params, r.m, r.v, r.hp, r.state, mode=1, grad_io=r.grad_io,
                         loss_slabs=r.loss_slabs, loss_out=r.grad_io[P:], loss_scale=scale)
            g = r.grad_io.clone()
            gsum = g.clone()
            for _ in range(1, world):
                gsum = gsum + g
            FM.adam_slab(None, 0, 1.0, r.params, r.m, r.v, r.hp, r.state, mode=2, grad_io=gsum, img=r.img, pre=True)
            torch.cuda.synchronize()
            assert _error(hs[0]) == 0, step
            assert torch.equal(a.params, r.params), (step, float((a.params - r.params).abs().max()))
            assert torch.equal(a.m, r.m) and torch.equal(a.v, r.v), step
            assert torch.equal(a.img, r.img), step
            assert float(a.loss_out.item()) == float(gsum[P].item()), step
    finally:
        torch.cuda.synchronize()
        _destroy(hs)


def test_proxy_missing_peer_times_out():
    """No emulator: the peers never publish, the consumer's wall-clock bound expires (0.3 s) and the
    error word is set (XgmiComm.check raises on it); the launch drains instead of hanging."""
    import torch

    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.ops import fused_mlp as FM

    dev = torch.device("cuda", 0)
    P = FM.P_TOTAL
    B = 8192
    draws = generate_masks(B + 16, seed=4, planted=0.8, device=dev)
    a = FusedSmallMLP(dev, lr=2e-3, seed=1)
    hs = _comms(4, P + 1, 0.3)
    try:
        p0 = a.params.clone()
        nslab = a._partials(draws, B, 0, None, step=a.state)
        FM.adam_slab_xgmi(hs[0].value, a.slabs, nslab, 1.0 / B, a.params, a.m, a.v, a.hp, a.state, a.loss_slabs,
                          img=a.img, loss_out=a.loss_out, loss_scale=1.0 / B, pre=True)
        torch.cuda.synchronize()
        assert _error(hs[0]) == 1
        assert torch.equal(a.params, p0)  # no block applied Adam without its peers
    finally:
        torch.cuda.synchronize()
        _destroy(hs)
