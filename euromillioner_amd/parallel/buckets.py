"""Bucketed gradient all-reduce overlapped with backward (C1).

Design for one 8-GPU MI355X node (xGMI is point-to-point, 7 links x ~153 GB/s per
GPU; a ring all-reduce is per-link bound, t ~ 2(N-1)/N * S / 153 GB/s):

* parameters are packed, in *reverse* registration order (the order backward
  produces their gradients), into flat fp32 buckets of ~``bucket_mb`` MB; each
  parameter's ``.grad`` is a view into its bucket, so no gradient is ever copied;
* a ``register_post_accumulate_grad_hook`` counts finished parameters per bucket;
  when a bucket is complete its all-reduce is launched immediately
  (``async_op=True``: RCCL runs on its own stream while backward continues);
* :meth:`finish` waits for the outstanding handles and rescales by 1/world.

Bucket sizing: the small MLP (64 KB of grads) is one latency-bound bucket; the wide
MLP (136 MB bf16 / 273 MB fp32) gets ~11 x 25 MB buckets so the first all-reduces
(the 8192x62 output layer) start while the 8192x8192 layer's backward is still
running.  A 25 MB fp32 bucket costs ~0.29 ms on one 8-rank ring at link rate.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class GradBucketer:
    def __init__(self, module: torch.nn.Module, bucket_mb: float = 25.0, group=None, world: int | None = None,
                 grad_dtype: torch.dtype = torch.float32):
        self.group = group
        self.world = world if world is not None else (dist.get_world_size(group) if dist.is_initialized() else 1)
        params = [p for p in module.parameters() if p.requires_grad]
        cap = max(1, int(bucket_mb * (1 << 20) // torch.tensor([], dtype=grad_dtype).element_size()))
        self.buckets: list[dict] = []
        cur: list[torch.nn.Parameter] = []
        size = 0
        for p in reversed(params):
            if cur and size + p.numel() > cap:
                self._make_bucket(cur, size, grad_dtype)
                cur, size = [], 0
            cur.append(p)
            size += p.numel()
        if cur:
            self._make_bucket(cur, size, grad_dtype)
        self.param_bucket = {}
        for bi, b in enumerate(self.buckets):
            for p in b["params"]:
                self.param_bucket[p] = bi
        self.handles: list = []
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params]
        self.enabled = self.world > 1

    def _make_bucket(self, params, size, dtype):
        dev = params[0].device
        buf = torch.zeros(size, dtype=dtype, device=dev)
        off = 0
        for p in params:
            p.grad = buf[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.buckets.append({"params": params, "buf": buf, "pending": len(params), "launched": False})

    def zero_grad(self) -> None:
        for b in self.buckets:
            b["buf"].zero_()
            b["pending"] = len(b["params"])
            b["launched"] = False
            off = 0
            for p in b["params"]:  # re-attach the view if anything replaced .grad
                view = b["buf"][off:off + p.numel()].view_as(p)
                if p.grad is None or p.grad.data_ptr() != view.data_ptr():
                    p.grad = view
                off += p.numel()
        self.handles = []

    def _on_grad(self, p):
        b = self.buckets[self.param_bucket[p]]
        b["pending"] -= 1
        if b["pending"] == 0 and self.enabled and not b["launched"]:
            b["launched"] = True
            self.handles.append(dist.all_reduce(b["buf"], op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def finish(self) -> None:
        """Wait for every bucket's all-reduce; gradients become the global mean."""
        if not self.enabled:
            return
        for b in self.buckets:  # buckets whose params got no grad this step still must participate
            if not b["launched"]:
                b["launched"] = True
                self.handles.append(dist.all_reduce(b["buf"], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        for h in self.handles:
            h.wait()
        self.handles = []
        inv = 1.0 / self.world
        for b in self.buckets:
            b["buf"].mul_(inv)

    def flat_grads(self) -> list[torch.Tensor]:
        return [b["buf"] for b in self.buckets]

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()


def plan_panels(rows: int, K: int, bucket_elems: int, ncu: int, tile_m: int = 256, tile_n: int = 256
                ) -> list[tuple[int, int]]:
    """Row panels [r0, r1) of a [rows, K] weight gradient produced by a 256x256-tile GEMM, each
    all-reduced as soon as it is written.  A panel is a whole number of full waves of tiles (one tile
    per CU: a 768-row panel of an 8192^2 gradient would run 96 tiles on 256 CUs) and at least
    ``bucket_elems`` elements: 8192 x 8192 on 256 CUs gives four 2048-row (64 MB fp32) panels."""
    tiles_per_row = max(1, K // tile_n)
    wave_rows = tile_m * max(1, -(-ncu // tiles_per_row))
    want = max(wave_rows, bucket_elems // max(K, 1))
    per = -(-want // wave_rows) * wave_rows
    return [(r, min(rows, r + per)) for r in range(0, rows, per)]


class RangeAllReducer:
    """Async SUM all-reduce of ranges of one flat gradient as they become final (C1 for the GEMM
    trainer): :meth:`ready` launches ``[a, c)`` in buckets of at most ``bucket_elems``; with ``wire``
    (a bf16 twin of the flat buffer) and ``cast`` (fp32 -> bf16 into it) the buckets travel in bf16.
    :meth:`wait` completes every launched bucket.  Buckets go out in the order ranges become ready,
    which is the same on every rank (the backward schedule is deterministic)."""

    def __init__(self, flat: torch.Tensor, bucket_elems: int, group=None, wire: torch.Tensor | None = None,
                 cast=None):
        self.flat, self.bucket_elems, self.group = flat, max(1, int(bucket_elems)), group
        self.wire, self.cast = wire, cast
        if wire is not None:  # each bucket's cast needs a 16-B aligned fp32 start: whole multiples of 8
            self.bucket_elems = max(8, self.bucket_elems // 8 * 8)
        self.handles: list = []
        self.launched: list[tuple[int, int]] = []

    def ready(self, a: int, c: int) -> None:
        if self.wire is not None and a % 4:
            raise ValueError(f"bf16-wire range must start at a multiple of 4 elements (got {a})")
        for s0 in range(a, c, self.bucket_elems):
            s1 = min(c, s0 + self.bucket_elems)
            if self.wire is not None:
                buf = self.cast(self.flat[s0:s1], self.wire[s0:s1])
            else:
                buf = self.flat[s0:s1]
            self.handles.append(dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            self.launched.append((s0, s1))

    def wait(self) -> None:
        for h in self.handles:
            h.wait()
        self.handles = []
