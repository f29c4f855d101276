#!/usr/bin/env python3
"""Per-workgroup wall-clock timeline of the ONE-LAUNCH fused step (train + in-launch slab reduction + Adam,
``em_mlp_fused_step``) inside a 10-launch hipGraph, next to the two-launch step's time.  Needs a
FUSED_STAMPS=1 side library (EUROM_NATIVE_LIB; ``tools/build_variant.sh stamps -DFUSED_STAMPS=1``): the stamps
are s_memrealtime marks (100 MHz) at kernel entry, prologue done, loop done, slab written and epilogue done,
written to spare slab floats.  Prints the critical path after the slowest workgroup's loop:
  last loop end -> last slab written -> last epilogue end, and how many chunks each workgroup processed."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.ops import fused_mlp as FM

    B = int(os.environ.get("TL_B", str(1 << 20)))
    draws = generate_masks(B + 16, seed=1, planted=0.9)
    for fused in (True, False):
        m = FusedSmallMLP("cuda", lr=1e-3, fused_adam=fused)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m.step(draws, B)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(10):
                    m.step(draws, B)
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(30):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        per = e0.elapsed_time(e1) * 1e3 / 10
        nslab = max(1, min(m.slabs.shape[0], (B + 127) // 128, 256))
        sp = m.slabs[:nslab, FM.P_TOTAL + 128:FM.P_TOTAL + 134].contiguous()
        raw = sp[:, :5].view(torch.int32).cpu().numpy()
        t = raw.astype(np.int64) & 0xFFFFFFFF
        t -= t[:, 0].min()
        us = t / 100.0
        q = lambda a: "min %.1f med %.1f max %.1f" % (a.min(), np.median(a), a.max())
        line = (f"{'one-launch' if fused else 'two-launch'} B={B}: {per:.1f} us/step (graph); loop end {q(us[:, 2])};"
                f" slab written {q(us[:, 3])}")
        if fused:
            chunks = sp[:, 5].cpu().numpy()
            last = int(np.argmax(us[:, 2]))
            line += (f"; epilogue end {q(us[:, 4])}; last loop end -> last slab {us[:, 3].max() - us[:, 2].max():.2f}"
                     f" -> last epilogue end {us[:, 4].max() - us[:, 3].max():.2f}; chunks per WG "
                     f"{np.bincount(chunks.astype(int)).tolist()}; slowest WG {last} did {int(chunks[last])} chunk(s),"
                     f" its epilogue {us[last, 4] - us[last, 3]:.2f} us")
        print(line, flush=True)
        del m


if __name__ == "__main__":
    main()
