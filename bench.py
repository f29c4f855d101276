#!/usr/bin/env python3
"""Headline benchmark: samples/sec training the 3-layer MLP (62-in/62-out) + val acc.

BASELINE.json metric "samples/sec training 3-layer MLP (62-in/62-out) at 1/2/4/8
MI355X; val acc", config "3-layer MLP (62->128->62) bf16 on 1xMI355X, 1M-row
synthetic batch" (DP=N over RCCL for N>1).

* one process per GPU: under torchrun (``WORLD_SIZE`` set) this process is one rank; with
  ``--gpus N > 1`` and no ``WORLD_SIZE`` it launches N ranks itself
  (``euromillioner_amd/parallel/launch.py``: subprocesses, no GPU call in the parent, no exec)
  and exits with the first failing rank's code;
* DP gradient all-reduce: the xGMI one-shot reduction fused into Adam when the node passes its
  self-test, else RCCL ("nccl") all-reduce of the flat gradient;
* weak scaling: every rank trains on its own 1M-row batch per step (global batch = N x 1M);
* ONE task for every rank: one synthetic draw sequence (one seed, so one planted Markov map)
  of N x draws-per-gpu draws generated on the GPU; the first 70% is the training split and the
  last 30% the validation split (positional, as ``Main.java:83-84,103-104``); rank r generates and
  trains on the r-th contiguous shard of the training split and evaluates the r-th shard of the
  validation split (metrics summed over ranks);
* a timed step = fused fwd+loss+bwd launch, [all-reduce], fused Adam launch —
  the full optimizer step, nothing skipped;
* the steps replay from hipGraphs of ``--graph-steps`` consecutive steps (each node set a full
  step with its own data offset), so graph-launch gaps are paid once per chunk;
* warmup: the W steps, then more untimed steps until ``--warmup-ms`` (250 ms) of wall time has
  passed, because the GPU ramps its clock over the first ~100 ms of load (at 20 timed steps the
  window would otherwise measure the ramp: 137 vs 117 us per step); the JSON reports the extra
  steps as ``warmup_extra_steps``;
* K steps timed between barrier + synchronize on both sides, MAX over ranks; hipEvents around
  each graph replay give the median step and the slowest rank's median;
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
    """Same model/loss/optimizer in plain PyTorch (bf16 autocast or fp32 GEMMs via hipBLASLt) — comparison only."""

    # torch.optim.Adam (capturable=False) refuses hipGraph capture: the baseline runs eager launches
    no_graph = True

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
        self.bf16 = a.dtype == "bf16"  # fp32: plain fp32 GEMMs

    def step(self, off):
        FM = self.FM
        FM.onehot(self.draws, self.B, offset=off, which=0, out=self.x)
        FM.onehot(self.draws, self.B, offset=off, which=1, out=self.y)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.bf16):
            z = self.net(self.x[:, :62].float())
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


def _pg_choice(dist_backend: str, model: str) -> tuple[str, bool]:
    """(process-group backend, high-priority RCCL streams) for N > 1: the requested backend for every model
    (the fused MLP's fallback all-reduce and its control plane run on it); high priority only for the wide
    model's bucketed all-reduces beside the GEMMs, where it was measured."""
    backend = "nccl" if dist_backend == "nccl" else "gloo"
    return backend, backend == "nccl" and model == "mlp-wide"


def _parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")),
                    help="ranks (one per GPU); without a torchrun env, N > 1 launches N processes")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1 << 20, help="rows per GPU per step (1M)")
    ap.add_argument("--draws-per-gpu", type=int, default=1 << 24,
                    help="draws of the shared sequence per rank (rounded up to whole 4096-draw segments)")
    ap.add_argument("--loss", default="softmax", choices=["softmax", "bce"])
    ap.add_argument("--lr", type=float, default=3e-3)
    ap.add_argument("--planted", type=float, default=0.9)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--graph", type=int, default=1, help="replay the step from hipGraphs (needs a graph-safe step)")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="consecutive training steps captured per hipGraph (each a full fwd+bwd+Adam step); "
                         "0 = all timed steps up to 50 in one graph (one launch latency per chunk)")
    ap.add_argument("--graph-chunks", default="",
                    help="explicit hipGraph plan for the timed steps: comma-separated step counts summing to "
                         "--steps, launched back to back (e.g. 1,19)")
    ap.add_argument("--warmup-ms", type=float, default=250.0,
                    help="after the W warmup steps, keep replaying untimed warmup steps until this much wall "
                         "time has passed (the chip ramps its clock over the first ~100 ms of load; a training "
                         "run spends its life at the steady clock).  0 = exactly W warmup steps")
    ap.add_argument("--no-eval", action="store_true")
    ap.add_argument("--impl", default="fused", choices=["fused", "gemm", "torch"],
                    help="fused = our HIP kernels (headline: the fused train kernel for --model mlp, the GEMM engine "
                         "for mlp-wide); gemm = the per-layer GEMM engine for --model mlp too; torch = plain "
                         "PyTorch/hipBLASLt eager (comparison)")
    ap.add_argument("--model", default="mlp", choices=["mlp", "mlp-wide"],
                    help="mlp = 62->128->62 (headline, fused kernel); mlp-wide = 62->8192->8192->62 (GEMM path)")
    ap.add_argument("--hidden", default=None, help="GEMM-path hidden sizes, e.g. 8192,8192")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="compute dtype: bf16 (headline) or fp32 (exact fp32 MFMA: the fused fp32 train kernel "
                         "csrc/mlp_fused_f32.hip for --model mlp, the fp32 GEMM engine csrc/gemm_f32.hip otherwise)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (nccl = RCCL; gloo only to rehearse N ranks sharing one GPU)")
    ap.add_argument("--device-data-gb", type=float, default=0.0,
                    help="HBM-resident dataset: this many GiB of draw masks per GPU (replaces --draws-per-gpu); "
                         "the timed steps are spread over the whole training shard (no hipGraph: offsets "
                         "change per step).  -1 = fill the GPU: free HBM (torch.cuda.mem_get_info) minus "
                         "--headroom-gb")
    ap.add_argument("--headroom-gb", type=float, default=10.0,
                    help="--device-data-gb -1: GiB left free for the model, slabs and the evaluation")
    ap.add_argument("--accum", type=int, default=1,
                    help="mlp-wide: micro-batches of --batch per optimizer step (gradient accumulation; "
                         "the per-GPU batch of the step is batch * accum)")
    ap.add_argument("--comm-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="mlp-wide: gradient all-reduce wire dtype (bf16 halves the bytes; Adam state stays fp32)")
    ap.add_argument("--bucket-mb", type=float, default=25.0, help="mlp-wide: gradient bucket size")
    ap.add_argument("--comm", default="auto", choices=["auto", "xgmi", "rccl"],
                    help="DP gradient all-reduce of the fused path: xgmi = one-shot peer-memory reduction fused "
                         "into Adam (hipGraph-replayable); rccl = torch.distributed all_reduce; auto = xgmi if the "
                         "node passes its self-test")
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="self-launched multi-rank job: kill every rank after this many seconds")
    return ap.parse_args()


SEG = 4096  # device generator segment (a rank's shard starts on a segment boundary)


class _Shards:
    """One draw sequence of ``world * n_loc`` draws; positional 70/30 split; rank r's contiguous
    shard of each split (``parallel.dist.shard_range``)."""

    def __init__(self, n_loc: int, rank: int, world: int):
        from euromillioner_amd.parallel.dist import DistInfo, shard_range

        self.n_draws = n_loc * world
        self.n_samples = self.n_draws - 1  # sample t = (draw t -> draw t+1)
        self.margin = int(0.7 * self.n_samples)
        info = DistInfo(rank, world)
        self.train = shard_range(self.margin, info)  # sample range [a, b) of this rank
        va, vb = shard_range(self.n_samples - self.margin, info)
        self.val = (self.margin + va, self.margin + vb)

    @staticmethod
    def materialize(rng, seed, planted, dev):
        """Masks covering samples [a, b) (draws a .. b) -> (buffer, offset of sample a in it)."""
        from euromillioner_amd.data.device_gen import generate_masks, region

        a, b = rng
        first, n, skip = region(a, b + 1, SEG)
        return generate_masks(n, seed=seed, planted=planted, seg_len=SEG, device=dev, first=first), skip


def _params_identical(model, world: int):
    """world > 1: True iff every rank ends the timed window with bit-identical parameters (the DP
    invariant; after a comm fallback it also shows the rebuilt model stayed in lockstep).  Small models
    compare the whole vector, large ones a 64-bit digest of the bits."""
    if world == 1:
        return None
    import torch.distributed as dist

    ps = [p for p in (getattr(model, "params", None),) if isinstance(p, torch.Tensor)]
    if not ps and hasattr(model, "parameters"):
        ps = [p for p in model.parameters() if isinstance(p, torch.Tensor)]
    if not ps:
        return None
    flat = torch.cat([p.detach().reshape(-1).float() for p in ps])
    if flat.numel() > (1 << 20):  # digest: int64 sum of the fp32 bit patterns, position-weighted
        bits = flat.view(torch.int32).to(torch.int64)
        w = torch.arange(1, bits.numel() + 1, device=bits.device, dtype=torch.int64) % 1000003
        flat = torch.stack([bits.sum(), (bits * w).sum()]).to(torch.float64)
    got = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(got, flat)
    return all(torch.equal(got[0], g) for g in got[1:])


def main():
    a = _parse()
    from euromillioner_amd.parallel import launch

    try:
        world, must_spawn = launch.requested_world(a.gpus)
    except ValueError as e:
        raise SystemExit(f"bench.py: {e}")
    if must_spawn:
        # this process never touches the GPU: N children, rank 0's stdout is the job's stdout
        argv = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(launch.spawn(argv, world, timeout_s=a.launch_timeout, quiet_ranks=True))

    if a.model == "mlp-wide":
        # 256k rows per optimizer step: the GEMMs' M, large enough that the per-step fixed costs (Adam over
        # 68M parameters, the skinny first/last layers' reductions) stay ~2 % of the step; measured
        # 3.57 / 3.59 / 3.61 M samples/s at 64k / 128k / 256k on one box (profiles/r6/bench_wide_batch.txt)
        if a.batch == 1 << 20:
            a.batch = 1 << 18
        if a.draws_per_gpu == 1 << 24:
            a.draws_per_gpu = (1 << 20) * 3

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(torch.cuda.device_count(), 1)
    if local >= ndev:
        if world > 1 and a.dist_backend == "nccl":
            raise SystemExit(f"bench.py: {world} RCCL ranks need {world} GPUs (found {ndev}); "
                             "use --dist-backend gloo to rehearse ranks sharing a GPU")
        local %= ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        import datetime

        import torch.distributed as dist

        backend, high_prio = _pg_choice(a.dist_backend, a.model)
        if high_prio:
            from euromillioner_amd.parallel.dist import high_priority_comm

            high_priority_comm()
        if backend == "nccl":
            dist.init_process_group("nccl", timeout=datetime.timedelta(minutes=10), device_id=dev)
        else:
            dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=10))
        group = dist.group.WORLD
        if dist.get_world_size() != world:
            raise SystemExit("bench.py: process group size != WORLD_SIZE")

    from euromillioner_amd.data.device_gen import gb_to_draws
    from euromillioner_amd.models.mlp import FusedSmallMLP

    if a.device_data_gb < 0:  # fill the GPU: what is free now, minus the headroom, on every rank
        free_b, _ = torch.cuda.mem_get_info(dev)
        # the training shard (70 % of the sequence) is what stays resident while training
        gb = max(1.0, (free_b / 2**30 - a.headroom_gb) / 0.7)
        if world > 1:  # every rank the same shard size (the smallest free memory)
            t = torch.tensor([gb], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            gb = float(t.item())
        a.device_data_gb = gb
    n_loc = gb_to_draws(a.device_data_gb) if a.device_data_gb > 0 else a.draws_per_gpu
    n_loc = -(-n_loc // SEG) * SEG
    sh = _Shards(n_loc, rank, world)
    torch.cuda.synchronize()
    tg = time.perf_counter()
    draws, tr_skip = sh.materialize(sh.train, a.seed, a.planted, dev)
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - tg
    resident_gb = draws.numel() * draws.element_size() / 2**30
    if a.device_data_gb > 0:
        a.graph = 0  # per-step offsets walk the whole training shard

    B = a.batch
    gemm_engine = a.model == "mlp-wide" or a.impl == "gemm"
    if a.accum < 1 or (a.accum > 1 and not gemm_engine):
        raise SystemExit("--accum applies to --model mlp-wide (the fused kernel takes any batch directly)")
    BS = B * a.accum  # samples per GPU per optimizer step
    n_train = sh.train[1] - sh.train[0]
    if n_train < BS:
        raise SystemExit("dataset too small for the batch")

    n_off = max(1, (n_train - BS) // BS + 1)
    # device-data runs spread the warmup + timed steps over the whole training shard
    spread = max(1, n_off // max(1, a.steps + a.warmup)) if a.device_data_gb > 0 else 1

    def boff(i):
        return tr_skip + ((i * spread) % n_off) * BS
    sizes = (62, 128, 62)
    if gemm_engine:
        from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer

        hidden = tuple(int(h) for h in (a.hidden or ("8192,8192" if a.model == "mlp-wide" else "128")).split(","))
        sizes = (62,) + hidden + (62,)
        model = GemmMLPTrainer(sizes, dev, loss=a.loss, lr=a.lr, seed=a.seed, process_group=group,
                               bucket_mb=a.bucket_mb, comm_dtype=a.comm_dtype, dtype=a.dtype)
        model.broadcast_parameters()

        def step(i):
            return model.step(draws, B, offset=boff(i), accum=a.accum)
    elif a.impl == "fused":
        model = FusedSmallMLP(dev, loss=a.loss, lr=a.lr, seed=a.seed, process_group=group, comm=a.comm,
                              dtype=a.dtype)
        model.broadcast_parameters()

        def step(i):
            return model.step(draws, B, offset=boff(i))
    else:
        model = _TorchBaseline(dev, a, draws, B, group)

        def step(i):
            return model.step(boff(i))

    use_graph = bool(a.graph) and not getattr(model, "no_graph", False) and (
        world == 1 or getattr(model, "graph_safe", False))
    loss_t = None
    tw = time.perf_counter()
    # warmup: with hipGraphs, one eager step (first-launch setup) and the other W-1 as replays of the
    # 1-step graph right before the timed loop, so the GPU enters it warm; otherwise W eager steps
    for i in range(a.warmup if not use_graph else min(a.warmup, 1)):
        loss_t = step(i)
    torch.cuda.synchronize()
    comm_fallback = None
    if world > 1 and getattr(model, "comm", None) == "xgmi" and a.comm == "auto":
        # the fused xGMI exchange has passed its self-test; if its first real step still reports a peer
        # wait that timed out on any rank, every rank rebuilds on the captured RCCL step instead of
        # failing the run (collective decision, same seed -> same initial parameters)
        try:
            model.check_comm()
            bad = 0
        except Exception as e:  # noqa: BLE001 -- reported, then handled by the fallback
            print(f"bench.py: rank {rank}: xGMI step failed ({e}); falling back to RCCL", file=sys.stderr)
            bad = 1
        t = torch.tensor([bad], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if int(t.item()):
            model.close()
            model = FusedSmallMLP(dev, loss=a.loss, lr=a.lr, seed=a.seed, process_group=group, comm="rccl",
                                  dtype=a.dtype)
            model.broadcast_parameters()
            comm_fallback = "xgmi step error -> rccl"
            use_graph = bool(a.graph) and not getattr(model, "no_graph", False) and getattr(model, "graph_safe", False)
            for i in range(a.warmup if not use_graph else min(a.warmup, 1)):
                loss_t = step(i)
            torch.cuda.synchronize()
    extra_warm = 0

    def clock_warmup(fn, n_per_call):
        """Untimed extra warmup steps until --warmup-ms of wall time has passed since warmup began
        (reported as warmup_extra_steps); every rank runs the same count (rank 0's) so DP ranks stay
        in lockstep."""
        nonlocal extra_warm
        calls = 0
        while True:
            go = (time.perf_counter() - tw) * 1000.0 < a.warmup_ms
            if world > 1:  # rank 0 decides, so every rank runs the same steps (each one a collective)
                t = torch.tensor([1 if go else 0], device=dev)
                dist.broadcast(t, 0)
                go = bool(t.item())
            if not go:
                break
            fn()
            calls += 1
            torch.cuda.synchronize()
        extra_warm = calls * n_per_call
    if use_graph:
        # hipGraphs of C consecutive steps (distinct data offsets baked into the nodes): one graph
        # launch per C steps, so the ~19 us launch gap between graph replays (rocprof kernel trace,
        # profiles/README.md) is paid once per chunk instead of once per step.  Steps that do not
        # fill a chunk replay a 1-step graph.
        C = max(1, min(a.graph_steps if a.graph_steps > 0 else 50, a.steps))
        chunks = [int(x) for x in a.graph_chunks.split(",") if x.strip()]
        if chunks and (sum(chunks) != a.steps or min(chunks) < 1):
            raise SystemExit("--graph-chunks must be positive step counts summing to --steps")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())

        def capture(n):
            nonlocal loss_t
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for c in range(n):
                    loss_t = step(c)
            return g
        with torch.cuda.stream(s):
            g_c = capture(C)
            g_1 = capture(1)
            g_by = {C: g_c, 1: g_1}
            for n in chunks:
                if n not in g_by:
                    g_by[n] = capture(n)
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(a.warmup - 1):
            g_1.replay()
        torch.cuda.synchronize()
        clock_warmup(g_c.replay, C)
        if chunks:
            C = max(chunks)
            plan = [(g_by[n], n) for n in chunks]
        else:
            plan = [(g_c, C)] * (a.steps // C) + [(g_1, 1)] * (a.steps % C)
        runs = [(lambda g=g: g.replay(), n) for g, n in plan]
    else:
        wi = iter(range(a.warmup, 1 << 62))
        clock_warmup(lambda: step(next(wi)), 1)
        runs = [(lambda i=i: step(i), 1) for i in range(a.steps)]

    ev0 = [torch.cuda.Event(enable_timing=True) for _ in runs]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in runs]
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k, (fn, _) in enumerate(runs):
        ev0[k].record()
        fn()
        ev1[k].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    ms = (t1 - t0) * 1000.0 / a.steps
    step_ms = sorted(e0.elapsed_time(e1) / n for e0, e1, (_, n) in zip(ev0, ev1, runs))
    med = step_ms[len(step_ms) // 2] if step_ms else float("nan")
    if hasattr(model, "check_comm"):
        model.check_comm()  # an xGMI peer wait that timed out is an error, not a fast step
    params_identical = _params_identical(model, world)
    med_max = med
    if world > 1:
        t = torch.tensor([ms, med], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms, med_max = float(t[0].item()), float(t[1].item())
    if rank == 0 and (t1 - t0) < 0.05:
        print(f"bench.py: warning: timed window {1000 * (t1 - t0):.1f} ms < 50 ms; use more --steps for a "
              "stable number", file=sys.stderr)
    loss = float(loss_t.reshape(-1)[0].item()) if loss_t is not None else float("nan")

    ev, ev_iid = {}, {}
    if not a.no_eval:
        del draws
        torch.cuda.empty_cache()
        va, vb = sh.val
        if a.device_data_gb > 0:  # cap the validation work (the full split can be tens of GiB)
            vb = min(vb, va + max(1, (1 << 24) // world))
        vdraws, v_skip = sh.materialize((va, vb), a.seed, a.planted, dev)
        ev = model.evaluate(vdraws, vb - va, offset=v_skip)
        del vdraws
        # the same model on iid draws (no planted structure): must sit at chance
        n_iid = -(-(1 << 20) // (world * SEG)) * SEG  # per rank
        iid = _Shards.materialize((rank * n_iid, (rank + 1) * n_iid), a.seed + 777, 0.0, dev)[0]
        ev_iid = model.evaluate(iid, n_iid, offset=0)

    value = BS * world / (ms / 1000.0)
    desc = "mlp " + "->".join(str(x) for x in sizes) + " relu, " + (
        "grouped softmax-CE" if a.loss == "softmax" else "sigmoid-BCE")
    extra = {}
    if gemm_engine:
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
            "warmup_extra_steps": extra_warm,
            "warmup_min_ms": a.warmup_ms,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": ("synthetic, generated on the GPU: one seeded Euromillions draw sequence of %d draws "
                     "(%d per GPU: %.1f GiB logical%s), planted Markov p=%.2f, shared by all ranks; positional "
                     "70/30 split, contiguous shard per rank; random-init weights"
                     % (sh.n_draws, n_loc, n_loc * 8 / 2**30,
                        "; the %.1f GiB training shard HBM-resident, the validation span regenerated and capped "
                        "at 16M draws" % resident_gb if a.device_data_gb > 0 else "", a.planted)),
            "config": {"model": desc,
                       "global_batch": BS * world, "seq_len": 1, "parallelism": f"dp{world}",
                       "per_gpu_batch": BS, "optimizer": "adam", "hipgraph": use_graph,
                       "engine": (("gemm_f32" if a.dtype == "fp32" else "gemm") if gemm_engine
                                  else a.impl + ("_f32" if a.dtype == "fp32" else "")),
                       "graph_steps": C if use_graph else 0,
                       "grad_allreduce": getattr(model, "comm", "rccl" if world > 1 else "none"),
                       "comm_fallback": comm_fallback,
                       "params_identical_across_ranks": params_identical,
                       **({"comm_dtype": a.comm_dtype, "bucket_mb": a.bucket_mb} if a.model == "mlp-wide" else {}),
                       "dist_backend": a.dist_backend if world > 1 else None},
            "ms_per_step_median": med,
            "ms_per_step_max_rank": med_max,
            "train_loss_last": loss,
            "val": ev,
            "val_iid": ev_iid,
            "datagen": {"draws": n_loc, "seconds": gen_s, "gb_per_s": resident_gb * 2**30 / max(gen_s, 1e-9) / 1e9,
                        "steps_spread": spread, "resident_train_gb": resident_gb,
                        "logical_sequence_gb_per_gpu": n_loc * 8 / 2**30},
            **extra,
        }
        print(json.dumps(out), flush=True)
    if hasattr(model, "close"):
        model.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
