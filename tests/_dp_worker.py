"""One rank of the multi-process data-parallel GPU test (tests/test_dp_gpu.py).

Backend from DP_BACKEND: "nccl" (RCCL; needs one GPU per rank) or "gloo" (rehearsal: ranks may
share a GPU).  Every rank holds the same global draw sequence and trains on its contiguous shard
(offset rank * B), so rank 0 can replay the whole global batch in one process as the reference.

Checks, printed as one JSON line:
* fused 62->128->62 step over the host all-reduce (comm="rccl") and over "auto" (xGMI when the
  node supports it): parameters bit-identical on every rank, equal to each other and to the
  single-process step on the global batch (up to summation order);
* GemmMLPTrainer (62->256->256->62) with bucketed async all-reduce: the same comparisons.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _identical(t: torch.Tensor, world: int) -> bool:
    allv = [torch.empty_like(t.cpu()) for _ in range(world)]
    dist.all_gather_object(allv, t.cpu())
    return all(torch.equal(allv[0], a) for a in allv)


def wide_case(dev, rank, world):
    """Wide GEMM trainer, data parallel with the bf16 wire and >= 3 async wgrad panels per hidden
    layer (panel_ncu pretends a 4-CU GPU): every rank ends bit-identical, and the parameters track a
    single-process run on the concatenated batch (the wire rounds the gradient to bf16, so Adam's
    per-element step may differ in magnitude, never by more than 2 lr per step)."""
    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer

    steps, B, lr = 3, 2048, 2e-3
    sizes = (62, 1024, 1024, 62)
    draws = generate_masks(world * B * steps + 16, seed=23, planted=0.8, device=dev)
    g = GemmMLPTrainer(sizes, dev, lr=lr, seed=0, process_group=dist.group.WORLD, bucket_mb=0.25,
                       comm_dtype="bf16")
    g.panel_ncu = 4
    g.broadcast_parameters()
    panels = g.wgrad_panels(1)
    for i in range(steps):
        g.step(draws, B, offset=(i * world + rank) * B)
    torch.cuda.synchronize()
    out = {"rank": rank, "world": world, "panels": len(panels), "wire_bf16": g.grads_bf16 is not None,
           "buckets": len(g.last_buckets), "identical": _identical(g.params, world)}
    if rank == 0:
        ref = GemmMLPTrainer(sizes, dev, lr=lr, seed=0)
        for i in range(steps):
            ref.step(draws, world * B, offset=i * world * B)
        torch.cuda.synchronize()
        d = (ref.params - g.params).abs()
        out.update(max_diff=float(d.max()), mean_diff=float(d.mean()), lr=lr, steps=steps)
    return out


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if os.environ.get("DP_CASE") == "wide":
        backend = os.environ.get("DP_BACKEND", "nccl")
        dev = torch.device("cuda", rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        out = wide_case(dev, rank, world)
        print("DP_RESULT " + json.dumps(out), flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return
    backend = os.environ.get("DP_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ndev)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer
    from euromillioner_amd.models.mlp import FusedSmallMLP

    out = {"rank": rank, "backend": backend, "devices": ndev}
    steps = 3

    # ---- fused small MLP
    B = 8192
    draws = generate_masks(world * B * steps + 16, seed=21, planted=0.8, device=dev)
    params = {}
    for kind in ("rccl", "auto"):
        m = FusedSmallMLP(dev, loss="softmax", lr=3e-3, seed=0, process_group=dist.group.WORLD, comm=kind)
        m.broadcast_parameters()
        out[f"fused_comm_{kind}"] = m.comm
        for i in range(steps):
            m.step(draws, B, offset=(i * world + rank) * B)
        torch.cuda.synchronize()
        m.check_comm()
        params[kind] = m.params.clone()
        out[f"fused_identical_{kind}"] = _identical(m.params, world)
        m.close()
    out["fused_rccl_vs_auto"] = float((params["rccl"] - params["auto"]).abs().max())
    if rank == 0:
        ref = FusedSmallMLP(dev, loss="softmax", lr=3e-3, seed=0)
        for i in range(steps):
            ref.step(draws, world * B, offset=i * world * B)
        torch.cuda.synchronize()
        out["fused_vs_single"] = float((ref.params - params["rccl"]).abs().max())

    # ---- GEMM-path MLP, bucketed async all-reduce (small buckets: several per layer)
    Bg = 2048
    sizes = (62, 256, 256, 62)
    g = GemmMLPTrainer(sizes, dev, lr=2e-3, seed=0, process_group=dist.group.WORLD, bucket_mb=0.1)
    g.broadcast_parameters()
    for i in range(steps):
        g.step(draws, Bg, offset=(i * world + rank) * Bg)
    torch.cuda.synchronize()
    out["gemm_identical"] = _identical(g.params, world)
    if rank == 0:
        ref = GemmMLPTrainer(sizes, dev, lr=2e-3, seed=0)
        for i in range(steps):
            ref.step(draws, world * Bg, offset=i * world * Bg)
        torch.cuda.synchronize()
        out["gemm_vs_single"] = float((ref.params - g.params).abs().max())
    print("DP_RESULT " + json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
