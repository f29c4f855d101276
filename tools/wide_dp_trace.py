#!/usr/bin/env python3
"""Overlap evidence for the wide MLP's data-parallel step (GemmMLPTrainer, 62->8192->8192->62).

Launches itself as 2 ranks (parallel/launch.py; gloo on a 1-GPU box: both ranks share the GPU, or
nccl on a node with >= 2 GPUs), profiles one training step per rank with torch.profiler after two
warmup steps, and writes from rank 0:
  * <out>/wide_dp_trace_rank0.json   chrome trace
  * <out>/wide_dp_overlap.md         the step's launch order: every GEMM kernel and every all-reduce
                                     launch (CPU-side ``all_reduce`` op) in time order, so one can see
                                     the 8192^2 layer's panel buckets going out before the last dgrad GEMM.

usage: python tools/wide_dp_trace.py [--backend gloo|nccl] [--batch 16384] [--out profiles]"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo", choices=["gloo", "nccl"])
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    ap.add_argument("--comm-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles"))
    a = ap.parse_args()
    from euromillioner_amd.parallel import launch

    if "WORLD_SIZE" not in os.environ:
        sys.exit(launch.spawn([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], 2, timeout_s=600))

    import torch
    import torch.distributed as dist
    from torch.profiler import ProfilerActivity, profile

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if a.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer

    B = a.batch
    masks = generate_masks(4 * world * B + 16, seed=3, planted=0.9, device=dev)
    tr = GemmMLPTrainer((62, 8192, 8192, 62), dev, process_group=dist.group.WORLD, bucket_mb=a.bucket_mb,
                        comm_dtype=a.comm_dtype)
    tr.broadcast_parameters()
    for k in range(2):
        tr.step(masks, B, offset=(k * world + rank) * B)
    torch.cuda.synchronize()
    dist.barrier()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        tr.step(masks, B, offset=(2 * world + rank) * B)
        torch.cuda.synchronize()
    dist.barrier()
    if rank == 0:
        os.makedirs(a.out, exist_ok=True)
        prof.export_chrome_trace(os.path.join(a.out, "wide_dp_trace_rank0.json"))
        import json

        trace = json.load(open(os.path.join(a.out, "wide_dp_trace_rank0.json")))
        ev = trace["traceEvents"] if isinstance(trace, dict) else trace
        gpu = {e["args"]["correlation"]: e for e in ev if e.get("cat") == "kernel" and "correlation" in e.get("args", {})}
        rows = []  # host program order: kernel launches (with their GPU span) and all-reduce enqueues
        for e in ev:
            if e.get("name") == "hipLaunchKernel":
                k = gpu.get(e["args"].get("correlation"))
                rows.append((e["ts"], "launch", e["args"].get("kernel", "")[:60],
                             (k["ts"], k["ts"] + k["dur"]) if k else None))
            elif e.get("name") == "c10d::allreduce_":
                rows.append((e["ts"], "all_reduce", "bucket", None))
        rows.sort(key=lambda r: r[0])
        t0 = min((r[3][0] for r in rows if r[3]), default=rows[0][0] if rows else 0)
        panels = tr.wgrad_panels(1)
        with open(os.path.join(a.out, "wide_dp_overlap.md"), "w", encoding="utf-8") as f:
            f.write(f"# Wide-MLP DP step: launch order (rank 0 of {world}, {a.backend}, batch {B}/rank, "
                    f"bucket {a.bucket_mb} MB, wire {a.comm_dtype})\n\n")
            f.write(f"8192^2 layer wgrad panels (rows): {panels}; buckets launched this step: "
                    f"{len(tr.last_buckets)}.  Host program order of the backward; an all-reduce enqueued "
                    "after a kernel waits on the GPU only for the kernels enqueued before it, so a bucket "
                    "listed before the last dgrad GEMM runs under it.\n\n")
            f.write("| # | host order | kernel GPU span (us) |\n|---|---|---|\n")
            for i, (ts, kind, name, span) in enumerate(rows):
                sp = f"{span[0] - t0:.0f} - {span[1] - t0:.0f}" if span else ""
                f.write(f"| {i} | {'**all_reduce**' if kind == 'all_reduce' else '`' + name + '`'} | {sp} |\n")
        print(f"wrote {a.out}/wide_dp_overlap.md ({len(rows)} events)")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
