#!/usr/bin/env python3
"""One-GPU budget of the DP=8 small-MLP gradient exchange (BASELINE.json configs[2]).

The pool's boxes have one GPU, so the 8-rank xGMI exchange of the fused 62->128->62 step is run as a
one-process proxy: rank 0 is the real model and its step is the real DP step, two launches (train
kernel -> ``em_adam_slab_xgmi``: each block reduces its 64-parameter slice of the slabs into the own
xGMI slot, raises its block flag, polls the 7 peers' block flags, sums 8 slices in rank order and
applies Adam), hipGraph-replayed like bench.py.  The 7 peers are buffers of this process on the same
device (``em_xgmi_connect_local``), played by ``em_xgmi_emulate_block_peers`` on a side stream beside
the consumer.  The timed "dpN" rows use its timing-only form (copy=0): one block raises all the peers'
block flags ``skew`` microseconds after the train kernel ends (the peers reaching the exchange later
than rank 0) and never waits on the consumer, so it adds no traffic of its own and cannot deadlock
when a replay runs it before the consumer.  The "dpN-copy" row uses the full form (block j waits for
rank 0's block flag j, copies the slice into the 7 peer slots, raises the peers' flag j: the traffic
real peers produce on their OWN GPUs), to show what that emulation costs on one device.

What it measures: the device cost of the 8-way exchange on top of the single-GPU step (7 extra slice
reads and block-flag polls inside the consumer), and how a late peer propagates into the step.  What it does not: xGMI link latency and bandwidth (the peer slots are local HBM here).  For
64 KB per peer over 7 links at ~50 GB/s effective that is ~1.3 us of transfer plus one hop of
~1-2 us; docs/DESIGN.md adds it to the budget.

Prints one JSON line per configuration.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.ops import _native as N
    from euromillioner_amd.ops import fused_mlp as FM
    from euromillioner_amd.parallel import xgmi as XG  # noqa: F401  (signatures)

    world = int(os.environ.get("XB_WORLD", "8"))
    B = int(os.environ.get("XB_B", str(1 << 20)))
    steps = 100
    dev = torch.device("cuda", 0)
    draws = generate_masks(4 * B + 16, seed=1, planted=0.9, device=dev)
    P = FM.P_TOTAL

    def make_comms():
        comms = []
        for _ in range(world):
            h = ctypes.c_void_p()
            rc = N.lib().em_xgmi_create(P + 1, 0.2, ctypes.byref(h))  # a protocol fault: error word, not a hang
            if rc != 0:
                raise SystemExit(f"em_xgmi_create failed ({rc})")
            comms.append(h)
        arr = (ctypes.c_void_p * world)(*[c.value for c in comms])
        N.call("em_xgmi_connect_local", comms[0], world, 0, arr)
        return comms

    def make_step(m, mode, skew_us, side):
        scale = 1.0 / (B * world)

        def step(off):
            nslab = m._partials(draws, B, off, None, check=False, step=m.state)
            if mode == "single":
                FM.adam_slab(m.slabs, nslab, 1.0 / B, m.params, m.m, m.v, m.hp, m.state, mode=0, img=m.img,
                             loss_slabs=m.loss_slabs, loss_out=m.loss_out, loss_scale=1.0 / B, pre=True)
                return
            ev = torch.cuda.Event()
            ev.record()
            side.wait_event(ev)
            if not mode.endswith("nowait"):
                with torch.cuda.stream(side):
                    N.call("em_xgmi_emulate_block_peers", h0, P // 64, P + 1, 1 if mode.endswith("copy") else 0,
                           float(skew_us), N.stream_handle(dev))
            FM.adam_slab_xgmi(h0, m.slabs, nslab, scale, m.params, m.m, m.v, m.hp, m.state, m.loss_slabs, img=m.img,
                              loss_out=m.loss_out, loss_scale=scale, pre=True)
            torch.cuda.current_stream().wait_stream(side)
        return step

    configs = ([("single", 0.0), ("dp%d-nowait" % world, 0.0)] + [("dp%d" % world, s) for s in (0.0, 2.0, 5.0, 10.0)]
               + [("dp%d-copy" % world, 0.0)])
    for rnd in range(int(os.environ.get("XB_ROUNDS", "2"))):
        for mode, skew in configs:
            m = FusedSmallMLP(dev, lr=1e-3, seed=0)
            comms = make_comms()
            h0 = comms[0].value
            if mode.endswith("nowait"):  # peers infinitely early: the consumer's own cost (lower bound)
                N.call("em_xgmi_emulate_block_peers", h0, P // 64, P + 1, 2, 0.0, N.stream_handle(dev))
                torch.cuda.synchronize()
            side = torch.cuda.Stream()
            step = make_step(m, mode, skew, side)
            step(0)  # eager first step (argument checks, LDS attributes)
            torch.cuda.synchronize()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    for i in range(10):
                        step((i % 4) * B)
            torch.cuda.current_stream().wait_stream(s)
            for _ in range(30):  # past the clock ramp
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(steps // 10):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / steps
            err = ctypes.c_int(0)
            N.call("em_xgmi_error", h0, ctypes.byref(err))
            torch.cuda.synchronize()
            print(json.dumps({"round": rnd, "mode": mode, "world": world if mode != "single" else 1,
                              "peer_skew_us": skew, "us_per_step": round(us, 2), "per_gpu_batch": B,
                              "xgmi_error": int(err.value), "loss": float(m.loss_out.item())}), flush=True)
            del g
            for c in comms:
                N.lib().em_xgmi_destroy(c)


if __name__ == "__main__":
    main()
