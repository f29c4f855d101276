"""Data parallelism across real processes on GPUs: RCCL at world 2/4/8 (one GPU per rank; skipped
with the reason on boxes with fewer GPUs, no edits needed on a full node) and a gloo rehearsal
that runs anywhere (ranks share the GPU).  Worker: tests/_dp_worker.py."""
import json
import os
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


def _run(world: int, backend: str, timeout: int = 180, case: str = ""):
    from euromillioner_amd.parallel.launch import host_store

    store, port = host_store(world)  # held by this process: rank 0 connects as a client (agent store)
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TORCHELASTIC_USE_AGENT_STORE="True", PYTHONPATH=ROOT, OMP_NUM_THREADS="2", DP_BACKEND=backend, DP_CASE=case,
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
        del store
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


@pytest.mark.parametrize("world,backend", [(1, "gloo"), (2, "gloo"), (2, "nccl"), (4, "nccl"), (8, "nccl")])
def test_wide_dp_panels_bf16_wire(world, backend):
    """Wide GEMM trainer (62->1024->1024->62) with the bf16 gradient wire and 4 async wgrad panels on
    the 1024x1024 layer: ranks bit-identical, tracking the single-process run on the concatenated batch.
    (2, gloo) runs two ranks on a one-GPU box (sharing the device): the GPU panel path with a real
    two-term bf16 all-reduce, which world 1 cannot exercise."""
    if backend == "nccl" and _ndev() < world:
        pytest.skip(f"RCCL world {world} needs {world} GPUs (this box has {_ndev()})")
    res = _run(world, backend, case="wide")
    for r in res:
        assert r["identical"] and r["wire_bf16"] and r["panels"] >= 3, r
        assert r["buckets"] >= r["panels"] + 2, r  # the hidden wgrad's panels + the other layers' ranges
    r0 = res[0]
    assert r0["max_diff"] <= 2 * r0["lr"] * r0["steps"] + 1e-6, r0
    assert r0["mean_diff"] <= 0.05 * r0["lr"], r0


def test_bench_xgmi_fault_falls_back_to_rccl():
    """bench.py's fallback: when the fused xGMI exchange passes its self-test but a rank then
    reports a timed-out peer wait, every rank rebuilds on the RCCL step.  Rank 1's wait is faulted by the
    test hook (EUROM_XGMI_FAULT_RANK=1); 2 ranks share the GPU over gloo.  The JSON must name the
    fallback, the step must run on the RCCL path, and the ranks must end bit-identical."""
    env = dict(os.environ, EUROM_XGMI_FAULT_RANK="1", PYTHONPATH=ROOT, OMP_NUM_THREADS="2",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "2",
                        "--no-eval", "--dist-backend", "gloo", "--batch", "65536", "--draws-per-gpu", str(1 << 20),
                        "--warmup-ms", "0", "--launch-timeout", "150"],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=170)
    assert p.returncode == 0, p.stdout[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, p.stdout[-3000:]
    d = json.loads(lines[-1])
    cfg = d["config"]
    assert cfg["comm_fallback"] == "xgmi step error -> rccl", cfg
    assert cfg["grad_allreduce"] == "rccl", cfg
    assert cfg["params_identical_across_ranks"] is True, cfg
    assert d["value"] > 0 and d["n_gpus"] == 2
