"""Process-group setup for one-process-per-GPU data parallelism (T4).

The reference declares Spark (``pom.xml:51-61``) but never uses it, and the north
star replaces Spark's ``ParameterAveragingTrainingMaster`` with synchronous gradient
all-reduce over RCCL (``torch.distributed`` backend ``"nccl"`` is RCCL on ROCm) on
one 8-GPU xGMI node.  CPU tests use ``gloo``.

* rendezvous from the torchrun env (``RANK``/``WORLD_SIZE``/``MASTER_ADDR``/...),
  always 127.0.0.1 for single-node runs;
* ``timeout`` so a dead peer raises instead of hanging;
* test-only fault injection: ``--fault-at-step k --fault-rank r`` makes rank r exit
  with code 17 at step k -- on the first attempt of a job only (a job restarted by
  ``parallel/launch.py --max-restarts`` or torchrun must not fail again at the same step).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str | None = None
    device: torch.device = torch.device("cpu")

    @property
    def is_dist(self) -> bool:
        return self.world > 1

    @property
    def group(self):
        return dist.group.WORLD if self.is_dist else None


def high_priority_comm() -> None:
    """RCCL's stream at high priority (before the process group is created): the bucketed gradient
    all-reduces of the wide trainer are issued while the backward GEMMs fill the chip, and a
    normal-priority collective queues behind them until the backward ends (the exposed tail in
    profiles/wide_dp_overlap.md).  Only the GEMM engine asks for it (``init(high_priority=True)``,
    bench.py --model mlp-wide): the fused small-MLP step and the GBDT run their collectives between
    launches, where the priority was never measured.  An explicit TORCH_NCCL_HIGH_PRIORITY
    in the environment wins."""
    os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")


def init(backend: str = "auto", timeout_s: float = 300.0, device: str = "auto",
         high_priority: bool = False) -> DistInfo:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available() and device != "cpu"
    dev = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(local)
    if world <= 1:
        return DistInfo(0, 1, 0, None, dev)
    be = backend if backend != "auto" else ("nccl" if use_cuda else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if not dist.is_initialized():
        kw = {"timeout": datetime.timedelta(seconds=timeout_s)}
        if be == "nccl":
            kw["device_id"] = dev
            if high_priority:
                high_priority_comm()
        dist.init_process_group(be, **kw)
    return DistInfo(rank, world, local, be, dev)


def barrier(info: DistInfo) -> None:
    if info.is_dist:
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.local_rank])
        else:
            dist.barrier()


def shutdown(info: DistInfo) -> None:
    if info.is_dist and dist.is_initialized():
        dist.destroy_process_group()


def maybe_inject_fault(step: int, info: DistInfo, at_step: int | None, at_rank: int | None) -> None:
    if at_step is None or step != int(at_step) or (at_rank is not None and int(at_rank) != info.rank):
        return
    if os.environ.get("EUROM_RESTART", "0") != "0" or os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") != "0":
        return  # a restarted job: the injected fault already happened
    os._exit(17)


def all_reduce_mean_(t: torch.Tensor, info: DistInfo) -> torch.Tensor:
    if info.is_dist:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t /= info.world
    return t


def broadcast_module_(module: torch.nn.Module, info: DistInfo, src: int = 0) -> None:
    """C2: identical initial parameters on every rank."""
    if not info.is_dist:
        return
    for p in list(module.parameters()) + list(module.buffers()):
        dist.broadcast(p.data, src=src)


def shard_range(n: int, info: DistInfo) -> tuple[int, int]:
    """Contiguous shard [a, b) of n items for this rank (sizes differ by at most 1)."""
    per, rem = divmod(n, info.world)
    a = info.rank * per + min(info.rank, rem)
    return a, a + per + (1 if info.rank < rem else 0)
