#!/usr/bin/env python3
"""One-GPU rehearsal of the wide-MLP DP overlap.

``run``: trains 62->8192->8192->62 at 64k rows per step three ways and prints one JSON line each:
  * ``none``     -- no communication (the single-GPU step);
  * ``sidecopy`` -- every gradient bucket, at the moment ``RangeAllReducer.ready`` would launch its
    all-reduce, gets a reduce-copy kernel on a side HIP stream (out = grad + peer over the bucket:
    2 reads + 1 write per element, the local HBM/CU footprint of a ring all-reduce's reduce step;
    xGMI bandwidth itself is not emulated), and the step waits for the side stream before Adam;
  * ``serial``   -- the same copies issued on the compute stream after the backward (no overlap).
``report TRACE.csv``: reads a rocprofv3 kernel trace of ``run`` (per-kernel stream ids and
timestamps) and prints, per mode, the wgrad-panel GEMM time with and without a concurrent side
copy and the fraction of side-copy time hidden under compute kernels.
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class SideCopy:
    """Stand-in for RangeAllReducer: same bucketing and launch points, a reduce-copy per bucket."""

    def __init__(self, flat, bucket_elems, side, peer, out, serial=False):
        import torch

        self.torch, self.flat, self.bucket, self.side = torch, flat, bucket_elems, side
        self.peer, self.out, self.serial = peer, out, serial
        self.launched, self.pending = [], []

    def ready(self, a, c):
        for s0 in range(a, c, self.bucket):
            s1 = min(c, s0 + self.bucket)
            self.launched.append((s0, s1))
            if self.serial:
                self.pending.append((s0, s1))
                continue
            ev = self.torch.cuda.Event()
            ev.record()
            self.side.wait_event(ev)
            with self.torch.cuda.stream(self.side):
                self.torch.add(self.flat[s0:s1], self.peer[s0:s1], out=self.out[s0:s1])

    def wait(self):
        for s0, s1 in self.pending:
            self.torch.add(self.flat[s0:s1], self.peer[s0:s1], out=self.out[s0:s1])
        self.torch.cuda.current_stream().wait_stream(self.side)


def run(steps: int = 20, B: int = 1 << 16, bucket_mb: float = 25.0):
    import torch

    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer

    dev = torch.device("cuda", 0)
    draws = generate_masks(B * 4 + 16, seed=3, planted=0.9, device=dev)
    m = GemmMLPTrainer((62, 8192, 8192, 62), dev, lr=1e-3, seed=0, bucket_mb=bucket_mb)
    side = torch.cuda.Stream()
    # the RCCL stream under TORCH_NCCL_HIGH_PRIORITY=1 (set by parallel.dist for the GEMM trainer): its
    # kernels are dispatched ahead of the GEMMs' when CUs free up, so the bucket queue does not back up
    side_hi = torch.cuda.Stream(priority=-1)
    peer = torch.randn(m.P + 1, device=dev)
    out = torch.empty_like(peer)
    modes = os.environ.get("WO_MODES", "none,sidecopy,sidecopy_hi,serial,none").split(",")
    for mode in modes:
        m.last_buckets = []
        m.comm_emulator = None if mode == "none" else (
            lambda flat, be, s=(mode == "serial"), st=(side_hi if mode == "sidecopy_hi" else side):
            SideCopy(flat, be, st, peer, out, serial=s))
        for i in range(3):
            m.step(draws, B, offset=(i % 4) * B)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.nvtx.range_push(mode) if hasattr(torch.cuda, "nvtx") else None
        t0 = time.perf_counter()
        e0.record()
        for i in range(steps):
            m.step(draws, B, offset=(i % 4) * B)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / steps
        print(json.dumps({"mode": mode, "ms_per_step": ms, "samples_per_s": B / ms * 1e3,
                          "buckets": len(m.last_buckets), "panels_layer1": len(m.wgrad_panels(1)),
                          "wall_s": time.perf_counter() - t0}), flush=True)
        time.sleep(0.5)  # a visible gap between the modes in the trace (report() splits on it)


def report(path: str):
    """Per mode (trace phases split at the 0.5 s sleeps): side-copy time and the fraction of it that
    ran concurrently with compute-stream kernels, and each compute kernel's time per step against
    the first no-communication phase (what the concurrent copies cost the GEMMs; the panelled wgrad
    is several launches per step in the communicating modes, one without)."""
    import csv

    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"])
                 for r in rows), key=lambda k: k[0])
    phases, cur = [], [ks[0]]
    for k in ks[1:]:
        if k[0] - cur[-1][1] > 200_000_000:
            phases.append(cur)
            cur = []
        cur.append(k)
    phases.append(cur)
    modes = os.environ.get("WO_MODES", "none,sidecopy,sidecopy_hi,serial,none").split(",")
    phases = [p for p in phases if len(p) > 50][-len(modes):]  # one phase per mode (setup kernels dropped)
    main = max(set(k[3] for k in ks), key=lambda s: sum(1 for k in ks if k[3] == s))
    

    def per_kernel(ph):  # compute-stream time per kernel name per optimizer step (Adam launches = steps)
        d = {}
        for k in ph:
            if k[3] == main:
                d.setdefault(k[2][:80], []).append(k[1] - k[0])
        steps = max(1, sum(len(v) for n, v in d.items() if "adam" in n))
        return {n: sum(v) / steps / 1e3 for n, v in d.items()}
    base = per_kernel(phases[0])
    for name, ph in zip(modes, phases):
        side = [k for k in ph if k[3] != main]
        comp = [k for k in ph if k[3] == main]
        hidden = 0
        for s0, s1, _, _ in side:
            for c0, c1, _, _ in comp:
                hidden += max(0, min(s1, c1) - max(s0, c0))
        side_t = sum(k[1] - k[0] for k in side)
        pk = per_kernel(ph)
        slow = {n: round(pk[n] / base[n], 3) for n in pk if n in base and base[n] > 100}
        print(json.dumps({"mode": name, "kernels": len(ph), "side_kernels": len(side), "side_us": side_t / 1e3,
                          "side_concurrent_frac": hidden / side_t if side_t else None,
                          "span_ms": (ph[-1][1] - ph[0][0]) / 1e6, "kernel_time_vs_none": slow}))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "report":
        report(sys.argv[2])
    else:
        run()
