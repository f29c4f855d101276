"""Gradient accumulation in the GEMM MLP trainer: accum micro-batches == one batch of the same samples."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sizes,B,accum", [((62, 512, 512, 62), 4096, 2), ((62, 1024, 62), 2048, 3)])
def test_accumulated_step_matches_single_batch(sizes, B, accum):
    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer

    masks = generate_masks(B * accum + 5000, seed=4, planted=0.8)
    a = GemmMLPTrainer(sizes, "cuda", seed=1)
    b = GemmMLPTrainer(sizes, "cuda", seed=1)
    la = a.step(masks, B * accum, offset=100)
    lb = b.step(masks, B, offset=100, accum=accum)
    torch.cuda.synchronize()
    assert abs(float(la) - float(lb)) < 1e-5 * max(1.0, abs(float(la)))
    ga, gb = a.grads[:a.P], b.grads[:b.P]
    err = (ga - gb).abs().max().item()
    assert err <= 2e-3 * ga.abs().max().item() + 1e-7, err
    # one more step with accumulation keeps the trainers close
    a.step(masks, B * accum, offset=100 + B * accum // 2)
    b.step(masks, B, offset=100 + B * accum // 2, accum=accum)
    assert (a.params - b.params).abs().max().item() < 5e-3


def test_cli_device_data_with_accumulation():
    """`euromillioner train --data-source device --accum 2` on the GEMM engine: learns the planted map."""
    from euromillioner_amd import config as C
    from euromillioner_amd.train import train

    cfg = C.build_config(None, {"model": "mlp", "device": "cuda", "data.source": "device", "data.n_draws": 200001,
                                "data.planted": 0.8, "data.seed": 3, "mlp.hidden": (256, 128), "mlp.batch": 4096,
                                "mlp.accum": 2, "mlp.steps": 150, "mlp.lr": 0.005, "mlp.eval_every": 0,
                                "log.level": "WARN"}, environ={})
    res = train(cfg)
    assert res["engine"] == "gemm"
    assert res["val"]["acc"] > res["val"]["trivial_acc"] and res["val"]["hits_main"] > 1.0, res["val"]


def test_cli_device_data_fused():
    from euromillioner_amd import config as C
    from euromillioner_amd.train import train

    cfg = C.build_config(None, {"model": "mlp", "device": "cuda", "data.source": "device", "data.n_draws": 300001,
                                "data.planted": 0.8, "mlp.batch": 8192, "mlp.steps": 150, "mlp.lr": 0.005,
                                "mlp.eval_every": 0, "log.level": "WARN"}, environ={})
    res = train(cfg)
    assert res["engine"] == "fused"
    assert res["val"]["acc"] > res["val"]["trivial_acc"] and res["val"]["hits_main"] > 1.0, res["val"]


@pytest.mark.parametrize("args", [["--device-data-gb", "0.25", "--steps", "3", "--warmup", "1"],
                                  ["--model", "mlp-wide", "--hidden", "512,512", "--batch", "8192", "--accum", "2",
                                   "--device-data-gb", "0.25", "--steps", "3", "--warmup", "1"]])
def test_bench_device_data_modes(args):
    """bench.py's HBM-resident-data and gradient-accumulation modes print one valid JSON line."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], capture_output=True, text=True,
                       timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["value"] > 0 and d["steps"] == 3 and d["datagen"]["draws"] > 0 and d["n_gpus"] == 1
    if "--accum" in args:
        assert d["config"]["per_gpu_batch"] == 16384 and d["accum"] == 2


def test_bench_two_ranks_share_one_task():
    """bench.py --gpus 2 (gloo, both ranks on this GPU) launches its own ranks, reports n_gpus 2, and --
    every rank training a shard of ONE planted sequence -- the averaged model beats the trivial
    all-zero predictor on validation (per-rank tasks averaged below it: ADVICE round 1)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = ["--gpus", "2", "--dist-backend", "gloo", "--steps", "40", "--warmup", "2", "--batch", "65536",
            "--draws-per-gpu", str(1 << 21)]
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], capture_output=True, text=True,
                       timeout=600, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2", d["config"]
    assert d["val"]["acc"] > d["val"]["trivial_acc"] + 0.01, d["val"]
