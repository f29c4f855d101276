"""Multi-process data parallelism on the CPU (gloo, 127.0.0.1): DP == single process,
bucketed == plain all-reduce, tree-parallel forest == single forest, fault injection
fails loudly instead of hanging, checkpoint resume continues exactly."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from euromillioner_amd.parallel.launch import host_store, rank_env

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "_dist_worker.py")


def _env(rank, world, port):
    env = rank_env(rank, world, port)  # the rendezvous store is hosted by this process (agent store)
    for k in ("LOCAL_WORLD_SIZE", "GROUP_RANK", "EUROM_LAUNCHED", "EUROM_RESTART"):
        env.pop(k)
    env.update(OMP_NUM_THREADS="1", PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    return env


def _launch(argv, world, timeout=240, cwd=None):
    # The test process hosts the TCPStore on a port it already holds (parallel/launch.py host_store): a
    # port picked free and bound later by rank 0 could be taken in between (the round-4 flake's
    # suspected cause).
    store, port = host_store(world)
    procs = [subprocess.Popen(argv, env=_env(r, world, port), cwd=cwd or ROOT, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out))
    del store
    return outs


def _ok(outs):
    """Fail with every failing rank's exit code and output tail (a list of 8 truncated outputs in one
    assert message hid the failing rank in round 4)."""
    bad = [(r, rc, out) for r, (rc, out) in enumerate(outs) if rc != 0]
    if bad:
        pytest.fail("\n".join(f"rank {r} exited {rc}:\n{out[-2500:]}" for r, rc, out in bad), pytrace=False)


def _train_argv(extra):
    return [sys.executable, "-m", "euromillioner_amd", "train", "--model", "mlp", "--device", "cpu",
            "--n-draws", "1201", "--planted", "0.7", "--seed", "5", "--eval-every", "0", "--log-level", "INFO"] + extra


def _params(path):
    from euromillioner_amd.ckpt import modelserializer as MS

    ck = MS.load(path)
    return ck["flat"], ck.get("m"), ck.get("v"), ck.get("extra", {})


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_equals_single_process(tmp_path, world):
    """Full-batch DP over `world` gloo ranks == one process on the whole batch."""
    single = str(tmp_path / "single.zip")
    multi = str(tmp_path / "multi.zip")
    # 1200 samples -> 840 train: divisible by 2 and 4, so every rank has the same local batch
    common = ["--steps", "6", "--batch", "840", "--lr", "0.01"]
    outs = _launch(_train_argv(common + ["--ckpt", single]), 1)
    assert outs[0][0] == 0, outs[0][1][-2000:]
    outs = _launch(_train_argv(common + ["--ckpt", multi, "--check-sync-every", "2"]), world)
    _ok(outs)
    a, b = _params(single), _params(multi)
    assert np.allclose(a[0], b[0], atol=2e-5), np.abs(a[0] - b[0]).max()  # reduction order differs
    assert np.allclose(a[1], b[1], atol=1e-6) and np.allclose(a[2], b[2], atol=1e-8)


@pytest.mark.parametrize("bucket_mb", ["0.01", "25"])
def test_bucketed_allreduce_equals_plain(tmp_path, bucket_mb):
    out = str(tmp_path / "b.json")
    res = _launch([sys.executable, WORKER, "buckets", out, bucket_mb], 2)
    _ok(res)
    r = json.load(open(out))
    assert r["max_err"] < 1e-6
    if bucket_mb == "0.01":
        assert r["n_buckets"] > 2  # several buckets, launched from the hooks during backward


def test_tree_parallel_forest_equals_single(tmp_path):
    from euromillioner_amd.data.draws import DrawSet
    from euromillioner_amd.models.forest import RandomForest, draw_features

    out = str(tmp_path / "f.npz")
    res = _launch([sys.executable, WORKER, "forest", out], 3)
    _ok(res)
    z = np.load(out, allow_pickle=False)
    ds = DrawSet.synthetic(n=900, seed=3, planted=0.5, calendar=False)
    X, Y, F = draw_features(ds.numbers)
    rf = RandomForest(n_trees=7, max_depth=4, seed=2, device="cpu").fit(X, Y, F)
    assert np.array_equal(z["feat"], rf.feat) and np.array_equal(z["value"], rf.value)


def test_fault_injection_fails_loudly(tmp_path):
    """Rank 1 dies at step 2 (exit 17); rank 0 must error out (non-zero) within the timeout."""
    argv = _train_argv(["--steps", "50", "--batch", "64", "--fault-at-step", "2", "--fault-rank", "1",
                        "--timeout", "30"])
    outs = _launch(argv, 2, timeout=200)
    assert outs[1][0] == 17, outs[1][1][-1500:]
    assert outs[0][0] != 0, outs[0][1][-1500:]


def test_resume_continues_exactly(tmp_path):
    full = str(tmp_path / "full.zip")
    part = str(tmp_path / "part.zip")
    base = ["--batch", "200", "--lr", "0.005"]  # minibatches with shuffling
    r = _launch(_train_argv(base + ["--steps", "12", "--ckpt", full]), 1)
    assert r[0][0] == 0, r[0][1][-2000:]
    r = _launch(_train_argv(base + ["--steps", "5", "--ckpt", part]), 1)
    assert r[0][0] == 0, r[0][1][-2000:]
    r = _launch(_train_argv(base + ["--steps", "12", "--ckpt", part, "--resume", part]), 1)
    assert r[0][0] == 0, r[0][1][-2000:]
    a, b = _params(full), _params(part)
    assert b[3]["step"] == 12
    assert np.allclose(a[0], b[0], atol=1e-6), np.abs(a[0] - b[0]).max()
    assert np.allclose(a[1], b[1], atol=1e-7)


def test_checkpoint_every_writes_intermediate(tmp_path):
    p = str(tmp_path / "c.zip")
    r = _launch(_train_argv(["--batch", "256", "--steps", "4", "--ckpt", p, "--ckpt-every", "2"]), 1)
    assert r[0][0] == 0, r[0][1][-2000:]
    assert _params(p)[3]["step"] == 4


def test_parameter_averaging_mode_stays_in_sync(tmp_path):
    """--avg-frequency k (Spark ParameterAveraging parity): local steps, averaged every k; the
    cross-rank checksum check (--check-sync-every) passes at every averaging point."""
    p = str(tmp_path / "avg.zip")
    outs = _launch(_train_argv(["--steps", "8", "--batch", "128", "--avg-frequency", "2",
                                "--check-sync-every", "2", "--ckpt", p]), 2)
    _ok(outs)
    assert _params(p)[3]["step"] == 8


def test_parameter_averaging_final_average(tmp_path):
    """steps % k != 0: the run still ends on one averaged model (final check_sync passes, and the
    checkpoint rank 0 writes is the average every rank holds)."""
    p = str(tmp_path / "avg7.zip")
    outs = _launch(_train_argv(["--steps", "7", "--batch", "128", "--avg-frequency", "3",
                                "--check-sync-every", "7", "--ckpt", p]), 2)
    _ok(outs)
    assert _params(p)[3]["step"] == 7


def _cli(args, timeout=400):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    return subprocess.run(args, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                          timeout=timeout)


def test_elastic_restart_resumes_bit_identical(tmp_path):
    """--dp 2 --max-restarts 1: rank 1 dies at step 5, the launcher restarts both ranks from the step-4
    checkpoint (--resume auto) and the job ends with exit 0 and the same parameters, bit for bit, as
    an uninterrupted run."""
    ref, got = str(tmp_path / "ref.zip"), str(tmp_path / "restarted.zip")
    common = ["--steps", "9", "--batch", "128", "--lr", "0.01", "--dp", "2", "--ckpt-every", "2"]
    r = _cli(_train_argv(common + ["--ckpt", ref]))
    assert r.returncode == 0, r.stdout[-3000:]
    r = _cli(_train_argv(common + ["--ckpt", got, "--fault-at-step", "5", "--fault-rank", "1",
                                   "--max-restarts", "1", "--timeout", "60"]))
    assert r.returncode == 0, r.stdout[-3000:]
    assert "restart 1/1" in r.stdout and "resumed from" in r.stdout
    a, b = _params(ref), _params(got)
    assert b[3]["step"] == 9
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y), np.abs(x - y).max()


def test_elastic_restart_with_parameter_averaging(tmp_path):
    """--avg-frequency 3 with --ckpt-every 2 takes checkpoints between averaging points;
    each averages first, so the restart from the step-4 checkpoint continues the interrupted run and
    the final parameters equal an uninterrupted run's, bit for bit."""
    ref, got = str(tmp_path / "ref.zip"), str(tmp_path / "restarted.zip")
    common = ["--steps", "9", "--batch", "128", "--lr", "0.01", "--dp", "2", "--ckpt-every", "2",
              "--avg-frequency", "3"]
    r = _cli(_train_argv(common + ["--ckpt", ref]))
    assert r.returncode == 0, r.stdout[-3000:]
    r = _cli(_train_argv(common + ["--ckpt", got, "--fault-at-step", "5", "--fault-rank", "1",
                                   "--max-restarts", "1", "--timeout", "60"]))
    assert r.returncode == 0, r.stdout[-3000:]
    assert "restart 1/1" in r.stdout
    a, b = _params(ref), _params(got)
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y), np.abs(x - y).max()


def test_no_restart_fails_loudly(tmp_path):
    """The same fault with --max-restarts 0: the job exits non-zero (rank 1's code 17)."""
    r = _cli(_train_argv(["--steps", "9", "--batch", "128", "--dp", "2", "--ckpt", str(tmp_path / "x.zip"),
                          "--ckpt-every", "2", "--fault-at-step", "5", "--fault-rank", "1", "--timeout", "60"]))
    assert r.returncode == 17, r.stdout[-3000:]
    assert "restart" not in r.stdout.replace("restarts", "")


def test_sync_check_detects_divergence(tmp_path):
    """Local steps that are not averaged yet diverge; the checker (step 2, long before the first
    averaging point and the end-of-run average) must fail loudly."""
    outs = _launch(_train_argv(["--steps", "4", "--batch", "128", "--avg-frequency", "1000",
                                "--check-sync-every", "2"]), 2)
    assert all(rc != 0 for rc, _ in outs)
    assert any("diverged" in o for _, o in outs)


def test_resume_auto(tmp_path):
    p = str(tmp_path / "auto.zip")
    base = ["--batch", "200", "--lr", "0.005", "--ckpt", p, "--resume", "auto"]
    r = _launch(_train_argv(base + ["--steps", "3"]), 1)  # nothing to resume: fresh start
    assert r[0][0] == 0, r[0][1][-2000:]
    r = _launch(_train_argv(base + ["--steps", "6"]), 1)
    assert r[0][0] == 0 and "resumed from" in r[0][1]
    assert _params(p)[3]["step"] == 6


@pytest.mark.parametrize("objective", ["reg:logistic", "multi:softprob"])
def test_data_parallel_gbdt_equals_single(tmp_path, objective):
    """C4: histogram all-reduce over 2 ranks == one process on the concatenated rows (multi-class:
    num_class inferred from the global label maximum, mlogloss from global row sums)."""
    from euromillioner_amd import config as C
    from euromillioner_amd.data.draws import DrawSet
    from euromillioner_amd.models.gbdt import GBDT
    from euromillioner_amd.parallel.dist import DistInfo, shard_range
    from euromillioner_amd.pipeline import gbdt_dataset

    out = str(tmp_path / "g.npz")
    res = _launch([sys.executable, WORKER, "gbdt", out, objective], 2)
    _ok(res)
    z = np.load(out, allow_pickle=False)
    ds = DrawSet.synthetic(n=700, seed=4, planted=0.6, calendar=True)
    X, Y, _ = gbdt_dataset(ds, C.RunConfig())
    Y = Y[:, :6]
    if objective.startswith("multi:"):
        Y = np.where(Y.any(1), np.argmax(Y, 1) + 1, 0).astype(np.float64)
        for lo, hi in (shard_range(500, DistInfo(1, 2)), [500 + v for v in shard_range(200, DistInfo(1, 2))]):
            Y[lo:hi] = np.minimum(Y[lo:hi], 5)
    m = GBDT(eta=0.5, max_depth=3, gamma=0.5, min_child_weight=0.5, nround=8, backend="numpy", objective=objective)
    m.fit(X[:500], Y[:500], evals={"test": (X[500:], Y[500:])})
    if objective.startswith("multi:"):
        assert m.num_class == 7 and z["leaf"].shape == m.trees.leaf.shape
    assert np.array_equal(z["feat"], m.trees.feat) and np.array_equal(z["sbin"], m.trees.sbin)
    assert np.allclose(z["leaf"], m.trees.leaf, atol=1e-6)
    assert np.allclose(z["hist"], [h["test"] for h in m.history], atol=1e-6)


def test_cli_pipeline_data_parallel(tmp_path):
    """`euromillioner run` under 2 ranks: DP boosting, only rank 0 prints the checkPredicts line."""
    argv = [sys.executable, "-m", "euromillioner_amd", "run", "--device", "cpu", "--n-draws", "400", "--nround", "4",
            "--workdir", str(tmp_path)]
    outs = _launch(argv, 2)
    _ok(outs)
    lines0 = [l for l in outs[0][1].splitlines() if l.strip() in ("true", "false")]
    lines1 = [l for l in outs[1][1].splitlines() if l.strip() in ("true", "false")]
    assert len(lines0) == 1 and not lines1
    assert '"world_size": 2' in outs[0][1]


def test_ckpt_at_averaging_points_keeps_trajectory(tmp_path):
    """with --avg-frequency k, checkpoints taken at averaging points (--ckpt-every a multiple
    of k) add no collective, so the run is bit-identical to the same run without intermediate
    checkpoints (a checkpoint between averaging points averages first: documented in train.py)."""
    a, b = str(tmp_path / "plain.zip"), str(tmp_path / "ckpt.zip")
    common = ["--steps", "8", "--batch", "128", "--lr", "0.01", "--avg-frequency", "2"]
    _ok(_launch(_train_argv(common + ["--ckpt", a]), 2))
    _ok(_launch(_train_argv(common + ["--ckpt", b, "--ckpt-every", "4"]), 2))
    pa, pb = _params(a), _params(b)
    for x, y in zip(pa[:3], pb[:3]):
        assert np.array_equal(x, y), np.abs(x - y).max()
