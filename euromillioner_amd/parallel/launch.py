"""Single-node rank launcher: ``bench.py --gpus N`` / ``euromillioner train --dp N`` without torchrun.

The north star replaces the reference's intended Spark runtime (``/root/reference/pom.xml:51-55``)
with one process per GPU over RCCL/xGMI.  ``torchrun`` is one way to start those processes; this
module is the other, so that ``--gpus N`` / ``--dp N`` mean what they say instead of silently running
one rank.

Rules that keep the launch safe on a GPU node:

* the parent never touches the GPU (no HIP call, no ``torch.cuda.is_available()``) and never
  ``exec``s — it starts N children with ``subprocess`` and waits;
* every child gets ``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``LOCAL_WORLD_SIZE`` and a 127.0.0.1
  rendezvous (``MASTER_ADDR``/``MASTER_PORT``) plus ``EUROM_LAUNCHED=1``;
* the rendezvous store is hosted by the parent (:func:`host_store`, as torchrun's agent does): it
  binds port 0 and keeps the socket, and the ranks connect as clients
  (``TORCHELASTIC_USE_AGENT_STORE=True``).  Picking a free port and letting rank 0 bind it later left
  a window in which another process (gloo's own pairwise connections, another job) could take the
  port; round 4's flaky 8-rank CPU test failed that way at rendezvous;
* the first child that fails (or the whole job passing ``timeout_s``) kills the others' process
  groups; the parent returns the failing child's exit code (124 for a timeout), never 0;
* elastic restart (``--max-restarts k``): after a rank failure the parent stops the
  job and starts ALL ranks again as fresh child processes (new rendezvous port), up to ``k`` times,
  with ``restart_argv`` (the trainers pass ``--resume auto``, so the new job continues from the last
  checkpoint).  Children see ``EUROM_RESTART=i`` (0 on the first attempt; test-only fault injection
  fires only there).  Each restart is logged; once the restarts are used up the job exits with the
  failing rank's code.  This replaces the reference's swallow-and-exit-0 handler
  (``/root/reference/src/main/java/com/euromillioner/Main.java:144-147``).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time

LAUNCHED_ENV = "EUROM_LAUNCHED"
RESTART_ENV = "EUROM_RESTART"


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def host_store(world: int, timeout_s: float = 900.0):
    """(store, port): a TCPStore server on 127.0.0.1 owned by the caller (pure CPU: no GPU is
    touched).  The port is bound from the start, so no other process can take it before the ranks
    connect; keep the returned store alive until the ranks have exited."""
    import datetime

    from torch.distributed import TCPStore

    store = TCPStore("127.0.0.1", 0, world, True, timeout=datetime.timedelta(seconds=timeout_s),
                     wait_for_workers=False)
    return store, int(store.port)


def rank_env(rank: int, world: int, port: int, base: dict | None = None, attempt: int = 0,
             agent_store: bool = True) -> dict:
    """Environment of rank ``rank`` of a ``world``-rank single-node job (``attempt``: restart index).
    ``agent_store``: the rendezvous store at ``port`` is hosted by the launcher (:func:`host_store`),
    so rank 0 connects to it as a client instead of binding the port itself."""
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port), LAUNCHED_ENV: "1", RESTART_ENV: str(attempt)})
    if agent_store:
        env["TORCHELASTIC_USE_AGENT_STORE"] = "True"
    else:
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
    # dmabuf IPC is the only kind the host driver supports (RCCL / xGMI peer buffers)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def requested_world(requested: int | None) -> tuple[int, bool]:
    """(world, must_spawn) for a ``--gpus``/``--dp`` request, checked against a torchrun env.

    * ``WORLD_SIZE`` set: we are a rank already; a request > 1 that differs is an error (1 is the
      flags' default, i.e. "not specified").
    * unset and ``requested > 1``: the caller must spawn ``requested`` ranks.
    """
    env_w = os.environ.get("WORLD_SIZE")
    req = int(requested) if requested else 0
    if req < 0:
        raise ValueError(f"rank count must be >= 1 (got {req})")
    if env_w is not None:
        w = int(env_w)
        if req > 1 and req != w:
            raise ValueError(f"requested {req} ranks but WORLD_SIZE={w} (launched by torchrun/launcher)")
        return w, False
    if req > 1:
        return req, True
    return 1, False


def restart_attempt() -> int:
    """Which (re)start of a self-launched job this process belongs to (0 = the first)."""
    try:
        return int(os.environ.get(RESTART_ENV, "0"))
    except ValueError:
        return 0


def spawn(argv: list[str], world: int, timeout_s: float = 3600.0, env: dict | None = None,
          quiet_ranks: bool = False, poll_s: float = 0.2, max_restarts: int = 0,
          restart_argv: list[str] | None = None) -> int:
    """Run ``argv`` as ``world`` ranks; return 0 iff every rank of the last attempt exited 0.

    ``quiet_ranks``: ranks > 0 get stdout discarded (their stderr still shows), so rank 0's
    output (e.g. the bench JSON line) is the only stdout of the job.
    ``max_restarts``: after a failed attempt, start every rank again (``restart_argv`` if given)
    at most this many times.  A job-level timeout is never retried.
    """
    if world < 1:
        raise ValueError("world must be >= 1")
    if max_restarts < 0:
        raise ValueError("max_restarts must be >= 0")
    t0 = time.monotonic()
    attempt = 0
    while True:
        cmd = argv if attempt == 0 or not restart_argv else restart_argv
        rc = _run_once(cmd, world, t0, timeout_s, env, quiet_ranks, poll_s, attempt)
        if rc == 0 or rc == 124 or attempt >= max_restarts:
            if rc != 0 and max_restarts > 0 and rc != 124:
                sys.stderr.write(f"[launch] giving up after {attempt} restart(s); exit {rc}\n")
            return rc
        attempt += 1
        sys.stderr.write(f"[launch] restart {attempt}/{max_restarts}: starting all {world} ranks again "
                         f"(previous attempt exited {rc})\n")
        sys.stderr.flush()


def _run_once(argv, world, t0, timeout_s, env, quiet_ranks, poll_s, attempt) -> int:
    store, port = host_store(world)  # a fresh store (and port) per attempt
    procs: list[subprocess.Popen] = []
    for r in range(world):
        out = subprocess.DEVNULL if (quiet_ranks and r > 0) else None
        procs.append(subprocess.Popen(argv, env=rank_env(r, world, port, env, attempt), stdout=out,
                                      start_new_session=True))
    rc_final = 0
    try:
        live = set(range(world))
        while live:
            for r in sorted(live):
                rc = procs[r].poll()
                if rc is None:
                    continue
                live.discard(r)
                if rc != 0 and rc_final == 0:
                    rc_final = rc if rc > 0 else 128 - rc  # -SIG -> 128+SIG
                    sys.stderr.write(f"[launch] rank {r} exited with {rc}; stopping the other ranks\n")
                    _kill_all(procs)
            if live and time.monotonic() - t0 > timeout_s:
                sys.stderr.write(f"[launch] job exceeded {timeout_s:.0f}s; stopping all ranks\n")
                _kill_all(procs)
                rc_final = 124
                break
            if live:
                time.sleep(poll_s)
    except KeyboardInterrupt:
        _kill_all(procs)
        raise
    finally:
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                _kill_group(p, signal.SIGKILL)
                p.wait()
        del store
    return rc_final


def _kill_group(p: subprocess.Popen, sig) -> None:
    if p.poll() is None:
        try:
            os.killpg(p.pid, sig)  # the child's own session (start_new_session=True)
        except ProcessLookupError:
            pass


def _kill_all(procs) -> None:
    for p in procs:
        _kill_group(p, signal.SIGTERM)
