"""Single-node rank launcher (parallel/launch.py): env wiring, failure exit codes, timeouts, and
``euromillioner train --dp N`` / ``bench.py --gpus N`` request checks (CPU only)."""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from euromillioner_amd.parallel import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _script(tmp_path, body: str) -> str:
    p = tmp_path / "child.py"
    p.write_text(body)
    return str(p)


def test_requested_world(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert launch.requested_world(1) == (1, False)
    assert launch.requested_world(None) == (1, False)
    assert launch.requested_world(4) == (4, True)
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert launch.requested_world(4) == (4, False)
    assert launch.requested_world(1) == (4, False)  # default request under torchrun
    with pytest.raises(ValueError):
        launch.requested_world(2)


def test_spawn_env_wiring(tmp_path, monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    out = tmp_path / "out"
    out.mkdir()
    child = _script(tmp_path, (
        "import json, os, sys\n"
        f"d = {str(out)!r}\n"
        "keys = ['RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT', 'EUROM_LAUNCHED',\n"
        "        'HSA_ENABLE_IPC_MODE_LEGACY']\n"
        "e = {k: os.environ.get(k) for k in keys}\n"
        "open(os.path.join(d, 'r' + e['RANK']), 'w').write(json.dumps(e))\n"))
    rc = launch.spawn([sys.executable, child], 3, timeout_s=60)
    assert rc == 0
    envs = [json.loads((out / f"r{r}").read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"] == [e["LOCAL_RANK"] for e in envs]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert {e["EUROM_LAUNCHED"] for e in envs} == {"1"}
    assert {e["HSA_ENABLE_IPC_MODE_LEGACY"] for e in envs} == {"0"}


def test_spawn_failure_stops_the_others(tmp_path):
    child = _script(tmp_path, (
        "import os, sys, time\n"
        "if os.environ['RANK'] == '1':\n"
        "    sys.exit(5)\n"
        "time.sleep(120)\n"))
    t0 = time.monotonic()
    rc = launch.spawn([sys.executable, child], 3, timeout_s=100)
    assert rc == 5
    assert time.monotonic() - t0 < 60  # the sleeping ranks were killed, not waited for


def test_spawn_timeout(tmp_path):
    child = _script(tmp_path, "import time\ntime.sleep(120)\n")
    rc = launch.spawn([sys.executable, child], 2, timeout_s=2)
    assert rc == 124


def test_spawn_quiet_ranks(tmp_path):
    child = _script(tmp_path, "import os\nprint('hello from', os.environ['RANK'])\n")
    r = subprocess.run([sys.executable, "-c",
                        "import sys; from euromillioner_amd.parallel import launch; "
                        f"sys.exit(launch.spawn([sys.executable, {child!r}], 3, quiet_ranks=True))"],
                       cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines() == ["hello from 0"]


def _cpu_env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PYTHONPATH=ROOT, OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    return env


def test_cli_dp_launches_ranks_and_matches_single(tmp_path):
    """``train --dp 2`` (no torchrun) starts 2 gloo ranks itself; full-batch DP == one process."""
    from euromillioner_amd.ckpt import modelserializer as MS

    base = [sys.executable, "-m", "euromillioner_amd", "train", "--model", "mlp", "--device", "cpu",
            "--n-draws", "1201", "--planted", "0.7", "--seed", "5", "--eval-every", "0",
            "--steps", "4", "--batch", "840", "--lr", "0.01"]
    one, two = str(tmp_path / "one.zip"), str(tmp_path / "two.zip")
    r1 = subprocess.run(base + ["--ckpt", one], cwd=ROOT, env=_cpu_env(), capture_output=True, text=True,
                        timeout=240)
    assert r1.returncode == 0, r1.stderr[-2000:]
    r2 = subprocess.run(base + ["--ckpt", two, "--dp", "2", "--check-sync-every", "2"], cwd=ROOT, env=_cpu_env(),
                        capture_output=True, text=True, timeout=240)
    assert r2.returncode == 0, r2.stderr[-2000:]
    assert "world=2" in r2.stderr + r2.stdout
    a, b = MS.load(one)["flat"], MS.load(two)["flat"]
    assert np.allclose(a, b, atol=2e-5)


def test_cli_dp_mismatch_with_torchrun_env_is_a_config_error():
    env = _cpu_env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-m", "euromillioner_amd", "train", "--model", "mlp", "--device", "cpu",
                        "--dp", "2"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2


def test_cli_dp_rank_failure_propagates():
    """A failing rank makes the launching CLI exit non-zero (fault injection on rank 1)."""
    r = subprocess.run([sys.executable, "-m", "euromillioner_amd", "train", "--model", "mlp", "--device", "cpu",
                        "--n-draws", "1201", "--steps", "50", "--batch", "64", "--dp", "2", "--fault-at-step", "2",
                        "--fault-rank", "1", "--timeout", "30"],
                       cwd=ROOT, env=_cpu_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 17, (r.returncode, r.stderr[-1500:])


def test_bench_gpus_mismatch_with_torchrun_env_fails():
    env = _cpu_env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_bench_process_group_backend_choice():
    """bench.py initialises the requested backend for every model at N > 1 (a round-5 edit had put the fused MLP
    on gloo under --dist-backend nccl, so its RCCL fallback would have run on gloo); high-priority RCCL streams
    only for the wide model's bucketed all-reduces."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench._pg_choice("nccl", "mlp") == ("nccl", False)
    assert bench._pg_choice("nccl", "mlp-wide") == ("nccl", True)
    assert bench._pg_choice("gloo", "mlp") == ("gloo", False)
    assert bench._pg_choice("gloo", "mlp-wide") == ("gloo", False)
