import io
import json

import numpy as np
import pytest

from euromillioner_amd import config as C
from euromillioner_amd import metrics as M


def test_defaults_are_reference_constants():
    cfg = C.RunConfig()
    assert cfg.gbdt_params() == {"booster": "gbtree", "eta": 1.0, "max_depth": 3, "predictor": "cpu_predictor",
                                 "objective": "reg:logistic", "subsample": 1.0, "silent": 1, "nthread": 6,
                                 "gamma": 1.0, "eval_metric": "logloss"}  # Main.java:113-126
    assert cfg.gbdt.nround == 500 and cfg.data.train_pct == 70 and cfg.data.label_column == 0
    assert cfg.data.to_date == "2020-06-14" and cfg.log.level == "INFO"


def test_precedence_file_env_cli(tmp_path):
    p = tmp_path / "c.json"
    p.write_text(json.dumps({"gbdt": {"eta": 0.5, "max_depth": 4}, "model": "rf"}))
    env = {"EUROM_GBDT__ETA": "0.25", "EUROM_MLP__HIDDEN": "64,32"}
    cfg = C.build_config(str(p), overrides={"gbdt.max_depth": 6}, environ=env)
    assert cfg.gbdt.eta == 0.25 and cfg.gbdt.max_depth == 6 and cfg.model == "rf"
    assert cfg.mlp.hidden == (64, 32)


def test_yaml_config(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("mlp:\n  lr: 0.01\n  batch: 4096\ndist:\n  dp: 2\n")
    cfg = C.build_config(str(p), environ={})
    assert cfg.mlp.lr == 0.01 and cfg.mlp.batch == 4096 and cfg.dist.dp == 2


def test_unknown_key_rejected():
    with pytest.raises(KeyError):
        C.build_config(overrides={"gbdt.nope": 1}, environ={})


def test_check_predicts_semantics():
    a = [[0.5], [0.25]]
    assert M.check_predicts(a, [[0.5], [0.25]])
    assert not M.check_predicts(a, [[0.5]])
    assert not M.check_predicts(a, [[0.5], [0.2500001]])
    assert M.check_predicts([[float("nan")]], [[float("nan")]])  # Arrays.equals: NaN == NaN
    assert not M.check_predicts([[0.0]], [[-0.0]])  # Arrays.equals: +0 != -0


def test_logloss_matches_definition():
    y = np.array([1, 0, 1])
    p = np.array([0.9, 0.2, 0.0])
    ref = -np.mean([np.log(0.9), np.log(0.8), np.log(1e-16)])
    assert abs(M.logloss(y, p) - ref) < 1e-12


def test_draw_metrics_trivial_and_perfect():
    rng = np.random.default_rng(0)
    Y = np.zeros((100, 62))
    for i in range(100):
        Y[i, rng.choice(50, 5, replace=False)] = 1
        Y[i, 50 + rng.choice(12, 2, replace=False)] = 1
    perfect = M.draw_metrics(Y * 10.0, Y)
    assert perfect["acc"] == 1.0 and perfect["exact"] == 1.0 and perfect["hits_main"] == 5
    assert abs(perfect["trivial_acc"] - 55 / 62) < 1e-12


def test_log4j_line_format():
    from euromillioner_amd import log as L

    buf = io.StringIO()
    L.setup("INFO", stream=buf)
    L.get("Main").warning("Could not access URL - x")
    line = buf.getvalue().strip()
    import re

    assert re.match(r"^\d{4}-\d\d-\d\d \d\d:\d\d:\d\d WARN  Main - Could not access URL - x$", line), line


@pytest.mark.parametrize("key,val", [("mlp.dtype", "fp16"), ("model", "cnn"), ("gbdt.objective", "rank:pairwise"),
                                     ("data.source", "web")])
def test_enumerated_fields_are_validated(key, val):
    with pytest.raises(ValueError):
        C.build_config(None, {key: val}, environ={})


def test_cli_rejects_bad_dtype_with_exit_2():
    from euromillioner_amd.cli import main

    assert main(["train", "--model", "mlp", "--dtype", "fp16", "--device", "cpu"]) == 2


def test_device_source_and_accum_validation():
    import pytest

    from euromillioner_amd import config as C

    with pytest.raises(ValueError):
        C.build_config(None, {"data.source": "device"}, environ={})  # needs n_draws or device_gb
    with pytest.raises(ValueError):
        C.build_config(None, {"mlp.batch": 1000, "mlp.accum": 3}, environ={})
    cfg = C.build_config(None, {"data.source": "device", "data.device_gb": 2.5, "mlp.accum": 4}, environ={})
    assert cfg.data.device_gb == 2.5 and cfg.mlp.accum == 4


def test_profile_dir_writes_a_chrome_trace(tmp_path):
    """--profile-dir exports a torch.profiler trace of the first profile_steps steps."""
    import os

    from euromillioner_amd.train import train

    cfg = C.build_config(None, {"model": "mlp", "device": "cpu", "data.n_draws": 400, "data.seed": 1,
                                "mlp.steps": 4, "mlp.batch": 64, "mlp.eval_every": 0, "log.level": "WARN",
                                "log.profile_dir": str(tmp_path), "log.profile_steps": 2}, environ={})
    train(cfg)
    files = [f for f in os.listdir(tmp_path) if f.endswith(".json")]
    assert files, os.listdir(tmp_path)
    assert os.path.getsize(os.path.join(tmp_path, files[0])) > 100


def test_fetch_jitter_flag_is_accepted():
    cfg = C.build_config(None, {"data.fetch_jitter_ms": "250"}, environ={})
    assert cfg.data.fetch_jitter_ms == 250
