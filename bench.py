#!/usr/bin/env python3
"""Headline benchmark: samples/sec training the 3-layer MLP (62-in/62-out) + val acc.

BASELINE.json metric "samples/sec training 3-layer MLP (62-in/62-out) at 1/2/4/8
MI355X; val acc", config "3-layer MLP (62->128->62) bf16 on 1xMI355X, 1M-row
synthetic batch" (DP=N over RCCL for N>1).

* one process per GPU (torchrun), RCCL ("nccl") all-reduce of the flat gradient;
* weak scaling: every rank trains on its own 1M-row batch per step (global batch
  = N x 1M), each rank reading its own shard of an HBM-resident synthetic draw
  sequence (planted Markov structure, seeded);
* a timed step = fused fwd+loss+bwd launch, [all-reduce], fused Adam launch —
  the full optimizer step, nothing skipped;
* K steps timed between barrier + synchronize on both sides, MAX over ranks;
* after timing, validation metrics on a held-out positional 30% split
  (outside the timed region).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1 << 20, help="rows per GPU per step (1M)")
    ap.add_argument("--draws-per-gpu", type=int, default=(1 << 24) + 1)
    ap.add_argument("--loss", default="softmax", choices=["softmax", "bce"])
    ap.add_argument("--lr", type=float, default=3e-3)
    ap.add_argument("--planted", type=float, default=0.9)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--graph", type=int, default=1, help="replay the step from a hipGraph (1 GPU)")
    ap.add_argument("--no-eval", action="store_true")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        import datetime

        import torch.distributed as dist

        dist.init_process_group("nccl", timeout=datetime.timedelta(minutes=10), device_id=dev)
        group = dist.group.WORLD

    from euromillioner_amd.data.synthetic import generate_draws
    from euromillioner_amd.models.mlp import FusedSmallMLP

    n_draws = a.draws_per_gpu
    nums, _ = generate_draws(n_draws, seed=a.seed + 1000 * rank, planted=a.planted, native=True)
    draws = torch.from_numpy(nums).to(dev)
    n_samples = n_draws - 1
    margin = int(0.7 * n_samples)
    B = a.batch
    if margin < B:
        raise SystemExit("dataset too small for the batch")

    model = FusedSmallMLP(dev, loss=a.loss, lr=a.lr, seed=a.seed, process_group=group)
    model.broadcast_parameters()
    n_off = max(1, (margin - B) // B)

    def step(i):
        return model.step(draws, B, offset=(i % n_off) * B)

    use_graph = bool(a.graph) and world == 1
    graph = None
    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    if use_graph:
        # offsets baked into graph nodes: capture n_off variants lazily would be heavy; capture a
        # ring of G graphs with distinct offsets and replay them round-robin.
        G = min(n_off, 8)
        graphs = []
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for gi in range(G):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    step(gi)
                graphs.append(g)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graph = graphs

        def run(i):
            graph[i % len(graph)].replay()
    else:
        def run(i):
            step(i)

    if world > 1:
        import torch.distributed as dist

        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        run(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    ms = (t1 - t0) * 1000.0 / a.steps
    if world > 1:
        t = torch.tensor([ms], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
    loss = float(model.loss_out.item() if group is None else model.grad_io[-1].item())

    ev = {}
    if not a.no_eval:
        ev = model.evaluate(draws, n_samples - margin, offset=margin)

    value = B * world / (ms / 1000.0)
    if rank == 0:
        out = {
            "metric": "samples/sec training 3-layer MLP (62-in/62-out)",
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (seeded Euromillions draws, planted Markov p=%.2f; random-init weights)" % a.planted,
            "config": {"model": "mlp 62->128->62 relu, grouped softmax-CE" if a.loss == "softmax" else
                       "mlp 62->128->62 relu, sigmoid-BCE",
                       "global_batch": B * world, "seq_len": 1, "parallelism": f"dp{world}",
                       "per_gpu_batch": B, "optimizer": "adam", "hipgraph": use_graph},
            "train_loss_last": loss,
            "val": ev,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
