#!/usr/bin/env python3
"""Is the fused 62->128->62 step bound by the chip's power/clock rather than by its instruction
stream?  The same launches (same kernels, same data, same control flow: the kernel has no
value-dependent branches) are timed with the model's random-init weights and with all weights zero
(lr = 0 in both, so nothing changes between steps).  Zero MFMA operands switch far fewer bits, so
if the step is power-bound the zero-weight arm holds a higher clock and runs faster at identical
cycles (MI355X_MICROARCH.md 'DVFS give-back' items 1, 3); if it is latency-bound both arms take the
same time.  Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
One JSON line per (round, arm)."""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.mlp import FusedSmallMLP

    B = 1 << 20
    dev = torch.device("cuda", 0)
    draws = generate_masks(4 * B + 16, seed=1, planted=0.9, device=dev)
    arms = {}
    for name in ("random", "zero"):
        m = FusedSmallMLP(dev, lr=0.0, seed=0)
        if name == "zero":
            m.params.zero_()
            m.FM.pack(m.params, m.img)
        m.step(draws, B, offset=0)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for i in range(20):
                    m.step(draws, B, offset=(i % 4) * B)
        torch.cuda.current_stream().wait_stream(s)
        arms[name] = (m, g)
    for rnd in range(3):
        for name, (m, g) in arms.items():
            for _ in range(40):  # ~70 ms of the same arm first: the clock settles to this workload
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"round": rnd, "arm": name, "us_per_step": round(e0.elapsed_time(e1) * 1e3 / 200, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
