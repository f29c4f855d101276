#!/usr/bin/env python3
"""Where the fused-MLP Adam launch's time goes (5.8 us per step, 17 MB of slabs).

Times ``em_adam_slab`` alone, replayed back to back from a hipGraph (device time per launch incl. the
kernel boundary), over the number of slabs it reduces (bytes read scale with nslab) and its modes:
mode 0 (slab reduce + Adam + bf16 image pack), mode 1 (slab reduce only, gradient to a buffer).  The
slope over nslab is the slab read rate, the intercept the fixed cost (launch, Adam, stores).

Prints one JSON line per configuration.
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.ops import fused_mlp as FM

    dev = torch.device("cuda", 0)
    m = FusedSmallMLP(dev, lr=1e-4, seed=0)
    m.slabs.normal_(0.0, 1e-3)
    m.loss_slabs.fill_(1.0)
    reps = 50
    junk = torch.empty(64 << 20, dtype=torch.float32, device=dev)  # 256 MB: evicts the L2s (and most of MALL)

    def timed(launch):
        launch()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(reps):
                    launch()
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        del g
        return e0.elapsed_time(e1) * 1e3 / (10 * reps)

    flush_us = timed(lambda: junk.fill_(0.5))
    print(json.dumps({"flush_us": round(flush_us, 2)}), flush=True)
    for nslab in (8, 32, 64, 128, 256):
        for mode in (0, 1):
            def one():
                if mode == 0:
                    FM.adam_slab(m.slabs, nslab, 1e-6, m.params, m.m, m.v, m.hp, m.state, mode=0, img=m.img,
                                 loss_slabs=m.loss_slabs, loss_out=m.loss_out, loss_scale=1e-6, pre=True)
                else:
                    FM.adam_slab(m.slabs, nslab, 1e-6, m.params, m.m, m.v, m.hp, m.state, mode=1, grad_io=m.grad_io,
                                 loss_slabs=m.loss_slabs, loss_out=m.grad_io[FM.P_TOTAL:], loss_scale=1e-6)

            def cold():
                junk.fill_(0.5)
                one()
            hot = timed(one)
            cold_us = timed(cold) - flush_us
            print(json.dumps({"nslab": nslab, "mode": mode, "mb_read": round(nslab * FM.P_TOTAL * 4 / 1e6, 2),
                              "us_hot": round(hot, 2), "us_after_flush": round(cold_us, 2)}), flush=True)


if __name__ == "__main__":
    main()
