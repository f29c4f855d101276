"""CLI integration: the default pipeline (== Main.main), subcommands, exit codes."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, env=None, timeout=600):
    e = dict(os.environ)
    e.update(env or {})
    e["PYTHONPATH"] = ROOT
    p = subprocess.run([sys.executable, "-m", "euromillioner_amd"] + args, capture_output=True, text=True,
                       timeout=timeout, env=e, cwd=ROOT)
    return p.returncode, p.stdout, p.stderr


def last_json(out):
    return json.loads([l for l in out.splitlines() if l.startswith("{")][-1])


def test_default_pipeline_small(tmp_path):
    rc, out, err = run(["--nround", "10", "--workdir", str(tmp_path), "--device", "cpu"])
    assert rc == 0, err + out
    lines = out.splitlines()
    assert "false" in lines  # Main.java:143 prints checkPredicts(train, validation) -> lengths differ
    res = last_json(out)
    assert res["n_draws"] == 1328 and res["n_train"] == int(0.7 * 1327) and res["target"] == "next-draw"
    assert os.path.exists(tmp_path / "emn.csv") and os.path.exists(tmp_path / "emn_validation.csv")
    assert "train-logloss" in out  # per-round watch-list logging (XGBoost4J format)


def test_reference_target_fails_like_xgboost():
    rc, out, err = run(["--target", "reference", "--nround", "2", "--device", "cpu"])
    assert rc == 3
    assert "label must be in [0,1]" in out + err


def test_reference_compat_squared_error():
    rc, out, err = run(["--target", "reference", "--objective", "reg:squarederror", "--eval-metric", "rmse",
                        "--nround", "5", "--reference-compat", "--device", "cpu"])
    assert rc == 0, err + out
    assert last_json(out)["check_predicts"] is False


def test_gen_and_csv_source(tmp_path):
    f = tmp_path / "d.csv"
    rc, out, _ = run(["gen", "--n", "500", "--planted", "0.9", "--out", str(f)])
    assert rc == 0 and json.loads(out)["draws"] == 500
    rc, out, err = run(["run", "--data-source", "csv", "--data-path", str(f), "--nround", "20", "--eta", "0.5",
                        "--device", "cpu"])
    assert rc == 0, err
    res = last_json(out)
    assert res["n_draws"] == 500 and res["val"]["acc"] > 0.9


def test_html_source():
    fix = os.path.join(ROOT, "tests", "fixtures", "results_table.html")
    rc, out, err = run(["--data-source", "html", "--data-path", fix, "--nround", "3", "--device", "cpu"])
    assert rc == 0, err
    assert last_json(out)["n_draws"] == 12


def test_missing_file_exit_code():
    rc, out, err = run(["--data-source", "csv", "--data-path", "/nonexistent.csv"])
    assert rc == 3


def test_bad_flag_value():
    rc, _, _ = run(["--nround", "abc"])
    assert rc == 2


def test_info():
    rc, out, _ = run(["info"])
    assert rc == 0 and "native" in json.loads(out)


def test_cli_train_rf_and_predict(tmp_path, capsys):
    from euromillioner_amd.cli import main

    ck = str(tmp_path / "rf.npz")
    rc = main(["train", "--model", "rf", "--device", "cpu", "--n-draws", "600", "--planted", "0.5",
               "--trees", "5", "--rf-max-depth", "4", "--ckpt", ck])
    assert rc == 0
    out = capsys.readouterr().out
    assert '"model": "rf"' in out
    rc = main(["predict", "--ckpt", ck, "--n-draws", "600", "--planted", "0.5"])
    assert rc == 0
    line = [l for l in capsys.readouterr().out.splitlines() if "*" in l and "{" not in l][0]
    main_nums, stars = line.split("*")
    assert len(main_nums.split()) == 5 and len(stars.split()) == 2


def test_cli_gbdt_checkpoint_predict(tmp_path, capsys):
    from euromillioner_amd.cli import main

    ck = str(tmp_path / "g.json")
    rc = main(["train", "--model", "gbdt", "--device", "cpu", "--n-draws", "300", "--nround", "5",
               "--ckpt", ck, "--workdir", str(tmp_path)])
    assert rc == 0
    rc = main(["predict", "--ckpt", ck, "--n-draws", "300"])
    assert rc == 0
    assert '"model": "gbdt"' in capsys.readouterr().out


def test_cli_predict_missing_checkpoint_is_data_error(tmp_path):
    from euromillioner_amd.cli import main

    assert main(["predict", "--ckpt", str(tmp_path / "nope.zip")]) == 3


def test_pipeline_cleans_temp_workdir(capsys):
    """D-h: without --workdir the split CSVs live in a temp dir that is removed afterwards."""
    import json as _json

    from euromillioner_amd.cli import main

    assert main(["run", "--device", "cpu", "--n-draws", "200", "--nround", "2"]) == 0
    out = capsys.readouterr().out
    js = [l for l in out.splitlines() if l.startswith("{")]
    assert js and _json.loads(js[-1])["workdir"] is None


def test_comm_dtype_flag_reaches_config_and_is_validated():
    import pytest

    from euromillioner_amd import cli
    from euromillioner_amd import config as C

    p = cli.build_parser()
    a = p.parse_args(["train", "--model", "mlp-wide", "--comm-dtype", "bf16", "--bucket-mb", "8"])
    cfg = cli._cfg_from_args(a)
    assert cfg.dist.comm_dtype == "bf16" and cfg.dist.bucket_mb == 8.0
    cfg.dist.comm_dtype = "fp16"
    with pytest.raises(ValueError, match="comm_dtype"):
        C.validate(cfg)


def test_next_draw_date_past_year_9999():
    """Long synthetic sequences (millions of draws) run past year 9999, where datetime.date cannot go:
    `predict` on a 2M-draw dataset failed with a TypeError before next_draw_date used datetime64 only."""
    import datetime as dt

    import numpy as np

    from euromillioner_amd.pipeline import next_draw_date

    for s in ["2004-02-13", "2011-05-06", "2011-05-10", "2011-05-13", "2026-10-16", "9999-12-30"]:
        d = dt.date.fromisoformat(s) + dt.timedelta(days=1) if s != "9999-12-30" else None
        if d is not None:
            while not (d.weekday() == 4 or (d.weekday() == 1 and d >= dt.date(2011, 5, 10))):
                d += dt.timedelta(days=1)
            assert next_draw_date(np.datetime64(s, "D")) == np.datetime64(d, "D"), s
    far = next_draw_date(np.datetime64("21173-01-26", "D"))
    assert far > np.datetime64("21173-01-26", "D") and (int(far.astype(np.int64)) + 3) % 7 in (1, 4)


def test_gen_accepts_n_draws_alias(tmp_path):
    """`gen --n-draws` (the name `train` uses) is the same as `gen --n`."""
    from euromillioner_amd import cli

    out = tmp_path / "d.csv"
    assert cli.main(["gen", "--n-draws", "300", "--out", str(out)]) == 0
    assert len([ln for ln in out.read_text().splitlines() if ln.strip()]) >= 300
