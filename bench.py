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


class _TorchBaseline:
    """Same model/loss/optimizer in plain PyTorch (bf16 autocast GEMMs via hipBLASLt) — comparison only."""

    def __init__(self, dev, a, draws, B, group):
        from euromillioner_amd.models.mlp import DrawMLP
        from euromillioner_amd.ops import fused_mlp as FM

        self.FM, self.draws, self.B, self.group, self.loss_name = FM, draws, B, group, a.loss
        self.net = DrawMLP((62, 128, 62), loss=a.loss, seed=a.seed, use_hip=False).to(dev)
        self.opt = torch.optim.Adam(self.net.parameters(), lr=a.lr)
        self.x = torch.empty(B, 64, dtype=torch.bfloat16, device=dev)
        self.y = torch.empty(B, 64, dtype=torch.bfloat16, device=dev)
        self.loss_out = torch.zeros(1, device=dev)
        self.grad_io = torch.zeros(1, device=dev)

    def step(self, off):
        FM = self.FM
        FM.onehot(self.draws, self.B, offset=off, which=0, out=self.x)
        FM.onehot(self.draws, self.B, offset=off, which=1, out=self.y)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            z = self.net(self.x[:, :62])
        loss = self.net.loss(z.float(), self.y[:, :62])
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        if self.group is not None:
            import torch.distributed as dist

            for p in self.net.parameters():
                dist.all_reduce(p.grad, group=self.group)
                p.grad /= dist.get_world_size(self.group)
        self.opt.step()
        self.loss_out = loss.detach().reshape(1)
        return self.loss_out

    def broadcast_parameters(self):
        pass

    def evaluate(self, draws, n, offset):
        from euromillioner_amd.data.draws import multi_hot  # noqa: F401
        from euromillioner_amd.models.losses import draw_metrics_torch

        b = min(n, 1 << 21)
        x = self.FM.onehot(draws, b, offset=offset, which=0)
        y = self.FM.onehot(draws, b, offset=offset, which=1)
        with torch.no_grad():
            z = self.net(x[:, :62].float())
        return draw_metrics_torch(z, y.float(), self.loss_name)


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
    ap.add_argument("--impl", default="fused", choices=["fused", "torch"],
                    help="fused = our HIP kernels (headline); torch = plain PyTorch/hipBLASLt eager (comparison)")
    ap.add_argument("--model", default="mlp", choices=["mlp", "mlp-wide"],
                    help="mlp = 62->128->62 (headline, fused kernel); mlp-wide = 62->8192->8192->62 (GEMM path)")
    ap.add_argument("--hidden", default=None, help="GEMM-path hidden sizes, e.g. 8192,8192")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (nccl = RCCL; gloo only to rehearse N ranks sharing one GPU)")
    ap.add_argument("--device-data-gb", type=float, default=0.0,
                    help="HBM-resident dataset: generate this many GiB of draw masks on the GPU "
                         "(csrc/datagen.hip) instead of --draws-per-gpu on the host; the timed steps "
                         "are spread over the whole training split (no hipGraph: offsets change per step)")
    ap.add_argument("--accum", type=int, default=1,
                    help="mlp-wide: micro-batches of --batch per optimizer step (gradient accumulation; "
                         "the per-GPU batch of the step is batch * accum)")
    ap.add_argument("--comm", default="auto", choices=["auto", "xgmi", "rccl"],
                    help="DP gradient all-reduce of the fused path: xgmi = one-shot peer-memory reduction fused "
                         "into Adam (hipGraph-replayable); rccl = torch.distributed all_reduce; auto = xgmi if the "
                         "node passes its self-test")
    a = ap.parse_args()
    if a.model == "mlp-wide":
        if a.batch == 1 << 20:
            a.batch = 1 << 16
        if a.draws_per_gpu == (1 << 24) + 1:
            a.draws_per_gpu = (1 << 20) * 3 + 1

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(torch.cuda.device_count(), 1)  # (identity on a node with >= N GPUs)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        import datetime

        import torch.distributed as dist

        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", timeout=datetime.timedelta(minutes=10), device_id=dev)
        else:
            dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=10))
        group = dist.group.WORLD

    from euromillioner_amd.data.synthetic import generate_draws
    from euromillioner_amd.models.mlp import FusedSmallMLP

    from euromillioner_amd.ops.fused_mlp import rows_to_masks

    gen_s = None
    if a.device_data_gb > 0:
        from euromillioner_amd.data.device_gen import gb_to_draws, generate_masks

        n_draws = gb_to_draws(a.device_data_gb)
        torch.cuda.synchronize()
        tg = time.perf_counter()
        draws = generate_masks(n_draws, seed=a.seed + 1000 * rank, planted=a.planted, device=dev)
        torch.cuda.synchronize()
        gen_s = time.perf_counter() - tg
        a.graph = 0  # per-step offsets walk the whole dataset
    else:
        n_draws = a.draws_per_gpu
        nums, _ = generate_draws(n_draws, seed=a.seed + 1000 * rank, planted=a.planted, native=True)
        draws = rows_to_masks(torch.from_numpy(nums).to(dev))  # device feature masks (8 B / draw)
    n_samples = n_draws - 1
    margin = int(0.7 * n_samples)
    B = a.batch
    if a.accum < 1 or (a.accum > 1 and a.model != "mlp-wide"):
        raise SystemExit("--accum applies to --model mlp-wide (the fused kernel takes any batch directly)")
    BS = B * a.accum  # samples per GPU per optimizer step
    if margin < BS:
        raise SystemExit("dataset too small for the batch")

    n_off = max(1, (margin - BS) // BS)
    # device-data runs spread the warmup + timed steps over the whole training split
    spread = max(1, n_off // max(1, a.steps + a.warmup)) if a.device_data_gb > 0 else 1

    def boff(i):
        return ((i * spread) % n_off) * BS
    sizes = (62, 128, 62)
    if a.model == "mlp-wide":
        from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer

        hidden = tuple(int(h) for h in (a.hidden or "8192,8192").split(","))
        sizes = (62,) + hidden + (62,)
        model = GemmMLPTrainer(sizes, dev, loss=a.loss, lr=a.lr, seed=a.seed, process_group=group)
        model.broadcast_parameters()

        def step(i):
            return model.step(draws, B, offset=boff(i), accum=a.accum)
    elif a.impl == "fused":
        model = FusedSmallMLP(dev, loss=a.loss, lr=a.lr, seed=a.seed, process_group=group, comm=a.comm)
        model.broadcast_parameters()

        def step(i):
            return model.step(draws, B, offset=boff(i))
    else:
        model = _TorchBaseline(dev, a, draws, B, group)

        def step(i):
            return model.step((i % n_off) * B)

    use_graph = bool(a.graph) and (world == 1 or getattr(model, "graph_safe", False))
    graph = None
    loss_t = None
    for i in range(a.warmup):
        loss_t = step(i)
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
                    loss_t = step(gi)
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
    if hasattr(model, "check_comm"):
        model.check_comm()  # an xGMI peer wait that timed out is an error, not a fast step
    if world > 1:
        t = torch.tensor([ms], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
    loss = float(loss_t.reshape(-1)[0].item()) if loss_t is not None else float("nan")

    ev, ev_iid = {}, {}
    if not a.no_eval:
        n_val = n_samples - margin if a.device_data_gb <= 0 else min(n_samples - margin, 1 << 24)
        ev = model.evaluate(draws, n_val, offset=margin)
        # the same model on iid draws (no planted structure): must sit at chance
        n_iid = min(1 << 20, n_samples - margin)
        iid_nums, _ = generate_draws(n_iid + 1, seed=a.seed + 777 + 1000 * rank, planted=0.0, native=True)
        iid = rows_to_masks(torch.from_numpy(iid_nums).to(dev))
        ev_iid = model.evaluate(iid, n_iid, offset=0)

    value = BS * world / (ms / 1000.0)
    desc = "mlp " + "->".join(str(x) for x in sizes) + " relu, " + (
        "grouped softmax-CE" if a.loss == "softmax" else "sigmoid-BCE")
    extra = {}
    if a.model == "mlp-wide":
        tf = model.flops_per_sample() * BS / (ms / 1000.0) / 1e12
        extra = {"tflops_per_gpu": tf, "flops_per_sample": model.flops_per_sample()}
        if a.accum > 1:
            extra.update({"micro_batch": B, "accum": a.accum})
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
            "data": ("synthetic (seeded Euromillions draws, planted Markov p=%.2f; random-init weights)" % a.planted
                     if a.device_data_gb <= 0 else
                     "synthetic, generated on the GPU: %.1f GiB of HBM-resident draw masks per GPU (%d draws, "
                     "planted Markov p=%.2f; random-init weights)" % (a.device_data_gb, n_draws, a.planted)),
            "config": {"model": desc,
                       "global_batch": BS * world, "seq_len": 1, "parallelism": f"dp{world}",
                       "per_gpu_batch": BS, "optimizer": "adam", "hipgraph": use_graph,
                       "grad_allreduce": getattr(model, "comm", "rccl" if world > 1 else "none")},
            "train_loss_last": loss,
            "val": ev,
            "val_iid": ev_iid,
            **extra,
        }
        if gen_s is not None:
            out["device_datagen"] = {"draws": n_draws, "gib": a.device_data_gb, "seconds": gen_s,
                                     "gb_per_s": n_draws * 8 / gen_s / 1e9, "steps_spread": spread}
        print(json.dumps(out))
    if hasattr(model, "close"):
        model.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
