"""End-to-end trainer on the GPU: every MLP engine, checkpoint resume, forest."""
import numpy as np
import pytest

from euromillioner_amd import config as C

pytestmark = pytest.mark.gpu


def _cfg(**over):
    base = {"model": "mlp", "device": "cuda", "data.n_draws": 6001, "data.planted": 0.8, "data.seed": 3,
            "mlp.eval_every": 0, "log.level": "WARN"}
    base.update(over)
    return C.build_config(None, base, environ={})


@pytest.mark.parametrize("hidden,lags,engine", [((128,), 1, "fused"), ((256, 128), 1, "gemm"), ((128,), 2, "torch")])
def test_engines_learn(hidden, lags, engine):
    from euromillioner_amd.train import train

    cfg = _cfg(**{"mlp.hidden": hidden, "data.lags": lags, "mlp.steps": 120, "mlp.batch": 1024, "mlp.lr": 0.005})
    res = train(cfg)
    assert res["engine"] == engine
    assert res["val"]["acc"] > res["val"]["trivial_acc"], res["val"]
    assert res["val"]["hits_main"] > 1.0


@pytest.mark.parametrize("hidden", [(128,), (192,)])
def test_gpu_resume_is_exact(tmp_path, hidden):
    from euromillioner_amd.ckpt import modelserializer as MS
    from euromillioner_amd.train import train

    full, part = str(tmp_path / "f.zip"), str(tmp_path / "p.zip")
    kw = {"mlp.hidden": hidden, "mlp.batch": 512, "mlp.lr": 0.003}
    train(_cfg(**kw, **{"mlp.steps": 10, "ckpt.path": full}))
    train(_cfg(**kw, **{"mlp.steps": 4, "ckpt.path": part}))
    train(_cfg(**kw, **{"mlp.steps": 10, "ckpt.path": part, "ckpt.resume": part}))
    a, b = MS.load(full), MS.load(part)
    assert np.allclose(a["flat"], b["flat"], atol=1e-6), np.abs(a["flat"] - b["flat"]).max()
    assert np.allclose(a["m"], b["m"], atol=1e-7)


def test_rf_on_gpu():
    from euromillioner_amd.train import train

    res = train(_cfg(**{"model": "rf", "rf.n_trees": 20, "rf.max_depth": 6}))
    assert res["backend"] == "hip" and res["trees"] == 20
    assert res["val"]["hits_main"] > 0.5
