"""One-shot intra-node all-reduce over xGMI peer memory (``csrc/xgmi.h`` / ``csrc/xgmi.hip``).

The flagship 62->128->62 step all-reduces a 64 KB gradient.  On one MI355X node the 8 GPUs
form a full xGMI mesh (7 point-to-point links per GPU), so instead of an RCCL ring (2(N-1)
latency-bound hops) every rank publishes its gradient in an IPC-shared, uncached HBM buffer
and the Adam kernel of every rank reads all N buffers directly — one hop over N-1 links in
parallel — summing them in rank order so parameters stay bit-identical across ranks.  No
host round trip and no collective launch: the whole DP step is two kernels (the train kernel, then
``em_adam_slab_xgmi``: slab reduction into the own slot, exchange and Adam) and replays from a
hipGraph.

The communicator is created collectively over an existing process group (gloo or RCCL; the
group only carries the 64-byte IPC handles and the go/no-go vote), self-tested against the
exact expected sum, and discarded — the caller falls back to RCCL — if any rank cannot open
its peers or the test fails.  Every wait inside a kernel is bounded by a wall-clock timeout
that raises an error word instead of hanging the GPU; :meth:`XgmiComm.check` turns it into an
exception.

Reference parity: the reference has no collectives (``Main.java:137-138`` is
single-process XGBoost); this is the C1 gradient all-reduce of the north star's DP config.
"""
from __future__ import annotations

import ctypes
import os
import socket

import torch
import torch.distributed as dist

from ..ops import _native as N

_v = ctypes.c_void_p
N.register_signatures({
    "em_xgmi_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_double, ctypes.POINTER(_v)]),
    "em_xgmi_handle": (ctypes.c_int, [_v, ctypes.c_char_p]),
    "em_xgmi_connect": (ctypes.c_int, [_v, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]),
    "em_xgmi_set_timeout": (ctypes.c_int, [_v, ctypes.c_double]),
    "em_xgmi_error": (ctypes.c_int, [_v, ctypes.POINTER(ctypes.c_int)]),
    "em_xgmi_capacity": (ctypes.c_int, [_v]),
    "em_xgmi_destroy": (ctypes.c_int, [_v]),
    "em_xgmi_stage": (ctypes.c_int, [_v, _v, ctypes.c_int, _v]),
    "em_xgmi_reduce": (ctypes.c_int, [_v, _v, ctypes.c_int, ctypes.c_float, _v]),
    "em_adam_slab_xgmi": (ctypes.c_int, [_v, _v, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int, _v, _v, _v,
                                         _v, _v, _v, _v, _v, ctypes.c_float, ctypes.c_int, ctypes.c_int, _v]),
    "em_xgmi_connect_local": (ctypes.c_int, [_v, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_v)]),
    "em_xgmi_emulate_peers": (ctypes.c_int, [_v, ctypes.c_int, ctypes.c_double, _v]),
    "em_xgmi_emulate_block_peers": (ctypes.c_int, [_v, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                                   _v]),
})

MAX_WORLD = 8  # one node (XG_MAXW in xgmi.h)
MAX_RANKS_PER_DEVICE = 2  # more ranks on one GPU: comm="auto" falls back to RCCL, comm="xgmi" raises
# Consumer blocks of a rank sharing its GPU: each spinning block holds a CU that the peer's train kernel
# (one 512-thread, 256-VGPR workgroup per CU) cannot use; 64 leave 192 CUs for it.
SHARED_DEVICE_BLOCKS = 64
DEFAULT_TIMEOUT_S = float(os.environ.get("EUROM_XGMI_TIMEOUT", "120"))


class XgmiError(RuntimeError):
    pass


def _vote_all(ok: bool, group) -> bool:
    """True iff every rank of ``group`` voted ok (object all-gather works on gloo and RCCL)."""
    votes = [None] * dist.get_world_size(group)
    dist.all_gather_object(votes, bool(ok), group=group)
    return all(bool(v) for v in votes)


class XgmiComm:
    """Handle to this rank's side of the xGMI communicator (see module docstring)."""

    def __init__(self, handle: int, world: int, rank: int, device: torch.device, cap: int,
                 ranks_per_device: int = 1):
        self.handle = handle
        self.world, self.rank, self.device, self.cap = world, rank, device, cap
        # > 1 when ranks share a GPU (tests on one-GPU boxes): the fused DP consumer then launches a
        # smaller grid (SHARED_DEVICE_BLOCKS) so its spinning blocks leave CUs for the peer's train kernel
        self.ranks_per_device = ranks_per_device

    @property
    def consumer_blocks(self) -> int:
        """Grid cap for ``em_adam_slab_xgmi`` (0 = one block per 64-parameter slice)."""
        return SHARED_DEVICE_BLOCKS if self.ranks_per_device > 1 else 0

    # ---------------------------------------------------------------- construction
    @classmethod
    def create(cls, group, device: torch.device, n_floats: int, timeout_s: float | None = None,
               verify: bool = True, required: bool = False):
        """Collective over ``group``.  Returns a verified communicator, or ``None`` when this
        node cannot use it (then the caller uses RCCL); ``required=True`` raises instead."""
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        reason = None
        if os.environ.get("EUROM_XGMI", "1").lower() in ("0", "off", "false", "no"):
            reason = "disabled by EUROM_XGMI=0"
        elif device.type != "cuda":
            reason = "not a GPU device"
        elif world > MAX_WORLD:
            reason = f"world {world} > {MAX_WORLD} (one node)"
        # identical decision on every rank: gather (host, device, local reason)
        me = (socket.gethostname(), int(device.index or 0), reason)
        allv = [None] * world
        dist.all_gather_object(allv, me, group=group)
        hosts = {h for h, _, _ in allv}
        reasons = [r for _, _, r in allv if r]
        per_dev = {}
        for h, d, _ in allv:
            per_dev[(h, d)] = per_dev.get((h, d), 0) + 1
        crowded = max(per_dev.values())
        if reasons:
            reason = reasons[0]
        elif len(hosts) != 1:
            reason = "ranks span several hosts"
        elif crowded > MAX_RANKS_PER_DEVICE:
            # every consumer kernel spins on its peers' flags while holding CUs; with more than two
            # processes on one device the peers' producers (whole-CU train kernels) are not
            # guaranteed to be scheduled meanwhile (docs/DESIGN.md §3, "ranks sharing a device")
            reason = f"{crowded} ranks share one device (at most {MAX_RANKS_PER_DEVICE})"
        else:
            for _, d, _ in allv:
                if d != me[1] and not torch.cuda.can_device_access_peer(me[1], d):
                    reason = f"no peer access cuda:{me[1]} -> cuda:{d}"
                    break
            reason = None if _vote_all(reason is None, group) else (reason or "a peer lacks P2P access")
        if reason:
            if required:
                raise XgmiError(f"xGMI all-reduce unavailable: {reason}")
            return None

        h = _v()
        t = DEFAULT_TIMEOUT_S if timeout_s is None else float(timeout_s)
        rc = N.lib().em_xgmi_create(int(n_floats), t, ctypes.byref(h))
        buf = ctypes.create_string_buffer(64)
        ok = rc == 0 and N.lib().em_xgmi_handle(h, buf) == 0
        handles = [None] * world
        dist.all_gather_object(handles, buf.raw if ok else None, group=group)
        ok = ok and all(x is not None for x in handles)
        if ok:
            ok = N.lib().em_xgmi_connect(h, world, rank, b"".join(handles)) == 0
        if not _vote_all(ok, group):
            if h.value:
                N.lib().em_xgmi_destroy(h)
            if required:
                raise XgmiError("xGMI all-reduce: IPC open failed on some rank")
            return None
        comm = cls(h.value, world, rank, device, N.lib().em_xgmi_capacity(h), ranks_per_device=crowded)
        if verify:
            comm.set_timeout(min(t, 20.0))  # ranks are in lock-step here (just voted)
            ok = comm.self_test()
            comm.set_timeout(t)
            if not _vote_all(ok, group):
                comm.close()
                if required:
                    raise XgmiError("xGMI all-reduce self-test failed")
                return None
        return comm

    # ---------------------------------------------------------------- ops
    def stage(self, src: torch.Tensor) -> None:
        """Producer: copy a local fp32 vector into this rank's next slot."""
        N.check_cuda(src, "src", torch.float32)
        N.call("em_xgmi_stage", self.handle, src.data_ptr(), src.numel(), N.stream_handle(src.device))

    def reduce(self, out: torch.Tensor, scale: float = 1.0) -> None:
        """Consumer: ``out = scale * sum_ranks(slot)`` (waits for every rank's producer)."""
        N.check_cuda(out, "out", torch.float32)
        N.call("em_xgmi_reduce", self.handle, out.data_ptr(), out.numel(), float(scale), N.stream_handle(out.device))

    def all_reduce_(self, t: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
        """In-place SUM (times ``scale``) of a small contiguous fp32 tensor across the node."""
        if t.numel() > self.cap:
            raise ValueError(f"{t.numel()} floats > communicator capacity {self.cap}")
        self.stage(t)
        self.reduce(t, scale)
        return t

    def error(self) -> int:
        e = ctypes.c_int(0)
        N.call("em_xgmi_error", self.handle, ctypes.byref(e))
        return int(e.value)

    def check(self) -> None:
        """Raise if any in-kernel wait on a peer timed out (synchronises with the device).
        ``EUROM_XGMI_FAULT_RANK=r`` (tests only) makes rank r report such a timeout, to drive the
        callers' fallbacks (bench.py rebuilds every rank on the RCCL step)."""
        fault = os.environ.get("EUROM_XGMI_FAULT_RANK")
        if fault is not None and fault.strip() != "" and int(fault) == self.rank:
            raise XgmiError(f"rank {self.rank}: injected xGMI peer-wait timeout (EUROM_XGMI_FAULT_RANK)")
        if self.error():
            raise XgmiError(f"rank {self.rank}: xGMI all-reduce timed out waiting for a peer "
                            f"(EUROM_XGMI_TIMEOUT={DEFAULT_TIMEOUT_S:g}s)")

    def set_timeout(self, seconds: float) -> None:
        N.call("em_xgmi_set_timeout", self.handle, float(seconds))

    def self_test(self) -> bool:
        """Two rounds (both slots) of an exactly-representable sum; True iff bit-exact."""
        n = min(self.cap, 1 << 15)
        idx = torch.arange(n, device=self.device, dtype=torch.float32)
        ok = True
        for rnd in range(2):
            x = (self.rank + 1 + 16 * rnd) + idx * 0.25
            want = sum((r + 1 + 16 * rnd) for r in range(self.world)) + idx * (0.25 * self.world)
            self.all_reduce_(x)
            torch.cuda.synchronize(self.device)
            ok = ok and self.error() == 0 and bool(torch.equal(x, want))
        return ok

    def close(self) -> None:
        if self.handle:
            N.lib().em_xgmi_destroy(_v(self.handle))
            self.handle = 0
