"""Gradient bucketing for the GEMM trainer's data parallelism (parallel/buckets.py), on the CPU:
the wgrad panel plan, and panel-by-panel range all-reduces (gloo, 2 ranks) == one all-reduce of the
whole gradient, in fp32 and over a bf16 wire."""
import os
import sys

import numpy as np

from euromillioner_amd.parallel import launch
from euromillioner_amd.parallel.buckets import plan_panels

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plan_panels_whole_tile_waves():
    p = plan_panels(8192, 8192, bucket_elems=25 << 18, ncu=256)
    assert p == [(0, 2048), (2048, 4096), (4096, 6144), (6144, 8192)]  # 256 tiles = one wave each
    # big buckets: several waves per panel
    assert plan_panels(8192, 8192, bucket_elems=8192 * 4096, ncu=256) == [(0, 4096), (4096, 8192)]
    # narrow K: a wave spans more rows; the last panel may be short
    p = plan_panels(4096, 1024, bucket_elems=1, ncu=256)
    assert p[0] == (0, 4096 if 4096 <= 256 * 64 else 256 * 64)
    for rows, K in ((8192, 8192), (6144, 2048), (512, 8192)):
        p = plan_panels(rows, K, 1 << 16, 256)
        assert p[0][0] == 0 and p[-1][1] == rows and all(a < b for a, b in p)
        assert all(p[i][1] == p[i + 1][0] for i in range(len(p) - 1))
        assert all((b - a) % 256 == 0 for a, b in p[:-1])


WORKER = r'''
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, {root!r})
from euromillioner_amd.parallel.buckets import RangeAllReducer, plan_panels

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
g = torch.Generator().manual_seed(7 + rank)
rows, K, B = 512, 96, 64
dz, x = torch.randn(rows, B, generator=g), torch.randn(K, B, generator=g)
flat = torch.zeros(rows * K + 10)
whole = (dz @ x.t()).reshape(-1).clone()
dist.all_reduce(whole)
out = {{}}
def aligned_cast(s, d):  # the HIP cast (em_cast_f32_bf16) rejects fp32 sources that are not 16-B aligned
    assert s.data_ptr() % 16 == 0, s.data_ptr()
    return d.copy_(s)
for wire_kind in ("fp32", "bf16"):
    flat.zero_()
    wire = torch.zeros_like(flat, dtype=torch.bfloat16) if wire_kind == "bf16" else None
    # an odd bucket size (what --bucket-mb 10.1 gives): the bf16 wire rounds it to whole 8-element groups
    red = RangeAllReducer(flat, bucket_elems=5000 if wire is None else 5003, wire=wire, cast=aligned_cast)
    assert wire is None or red.bucket_elems % 8 == 0
    gw = flat[:rows * K].view(rows, K)
    for r0, r1 in plan_panels(rows, K, 5000, ncu=2, tile_m=64, tile_n=32):
        gw[r0:r1] = dz[r0:r1] @ x.t()   # this panel is final ...
        red.ready(r0 * K, r1 * K)       # ... so its buckets go out now
    red.wait()
    got = (wire.float() if wire is not None else flat)[:rows * K]
    out[wire_kind] = float((got - whole).abs().max())
    out[wire_kind + "_buckets"] = len(red.launched)
    assert red.launched[0][0] == 0 and red.launched[-1][1] == rows * K
np.save(os.path.join({tmp!r}, "r%d.npy" % rank), np.array([out["fp32"], out["bf16"], out["fp32_buckets"]]))
dist.destroy_process_group()
'''


def test_panelled_range_allreduce_equals_whole(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER.format(root=ROOT, tmp=str(tmp_path)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    assert launch.spawn([sys.executable, str(script)], 2, timeout_s=120, env=env) == 0
    for r in range(2):
        fp32_err, bf16_err, nb = np.load(tmp_path / f"r{r}.npy")
        assert fp32_err < 1e-4  # same sums, split in ranges (gloo's 2-rank sum is order-free)
        assert bf16_err < 0.5  # entries up to ~50: bf16 wire rounding (~2^-8 relative) only
        assert nb > 4  # several panels, several buckets
