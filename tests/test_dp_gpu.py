"""Data parallelism across real processes on GPUs: RCCL at world 2/4/8 (one GPU per rank; skipped
with the reason on boxes with fewer GPUs, no edits needed on a full node) and a gloo rehearsal
that runs anywhere (ranks share the GPU).  Worker: tests/_dp_worker.py."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ndev() -> int:
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world: int, backend: str, timeout: int = 180):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PYTHONPATH=ROOT, OMP_NUM_THREADS="2", DP_BACKEND=backend,
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "_dp_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    res = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            assert p.returncode == 0, out[-3000:]
            line = [ln for ln in out.splitlines() if ln.startswith("DP_RESULT ")]
            assert line, out[-3000:]
            res.append(json.loads(line[-1][len("DP_RESULT "):]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return res


def _check(res, expect_xgmi: bool | None):
    for r in res:
        assert r["fused_comm_rccl"] == "rccl", r
        if expect_xgmi is not None:
            assert (r["fused_comm_auto"] == "xgmi") == expect_xgmi, r
        assert r["fused_identical_rccl"] and r["fused_identical_auto"], r
        assert r["fused_rccl_vs_auto"] < 1e-4, r
        assert r["gemm_identical"], r
    assert res[0]["fused_vs_single"] < 2e-4, res[0]
    assert res[0]["gemm_vs_single"] < 2e-3, res[0]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_data_parallel(world):
    if _ndev() < world:
        pytest.skip(f"RCCL world {world} needs {world} GPUs (this box has {_ndev()})")
    _check(_run(world, "nccl"), expect_xgmi=True)


def test_gloo_data_parallel_rehearsal():
    """Same worker, gloo group (host all-reduce of device tensors); ranks may share one GPU."""
    _check(_run(2, "gloo"), expect_xgmi=None)
