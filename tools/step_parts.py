#!/usr/bin/env python3
"""Where the headline step's time goes: hipGraphs of 10 back-to-back launches of (a) the fused train
kernel alone, (b) the Adam slab kernel alone, (c) the whole step (train + Adam), timed with events at
several batch sizes.  (c) - (a) - (b) is what the kernel boundaries cost; the slope of (a) over the
batch is the loop's marginal cost and its intercept the kernel's fixed cost."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed_graph(fn, reps: int = 10, iters: int = 20) -> float:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (iters * reps)  # us per launch


def main():
    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.ops import fused_mlp as FM

    draws = generate_masks((1 << 24) + 16, seed=1, planted=0.9)
    m = FusedSmallMLP("cuda", lr=1e-3)
    out = []
    sizes = [int(x) for x in os.environ.get("STEP_PARTS_B", "%d,%d,%d" % (1 << 20, 1 << 21, 1 << 22)).split(",")]
    for B in sizes:
        nslab = FM.train_partials(draws, B, m.img, m.slabs, m.loss_slabs, loss="softmax")
        lscale = 1.0 / B

        def train():  # as FusedSmallMLP.step runs it: the train kernel advances the Adam step counter
            FM.train_partials(draws, B, m.img, m.slabs, m.loss_slabs, loss="softmax", step=m.state)

        def adam():
            FM.adam_slab(m.slabs, nslab, 1.0 / B, m.params, m.m, m.v, m.hp, m.state, mode=0, img=m.img,
                         loss_slabs=m.loss_slabs, loss_out=m.loss_out, loss_scale=lscale, pre=True)

        def step():
            m.step(draws, B, offset=0)
        r = {"B": B, "train_us": timed_graph(train), "adam_us": timed_graph(adam), "step_us": timed_graph(step)}
        r["boundary_us"] = r["step_us"] - r["train_us"] - r["adam_us"]
        print(json.dumps(r), flush=True)
        out.append(r)
    if len(out) > 1:
        b0, b1 = out[0], out[-1]
        slope = (b1["train_us"] - b0["train_us"]) / ((b1["B"] - b0["B"]) / (1 << 20))
        print(json.dumps({"train_us_per_M": slope, "train_fixed_us": b0["train_us"] - slope}))


if __name__ == "__main__":
    main()
