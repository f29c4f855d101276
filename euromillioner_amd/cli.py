"""``euromillioner`` command line (T8).

The reference's CLI is "run with no arguments": ``Main.main`` ignores ``args`` and
runs the whole pipeline (``Main.java:35``).  Here:

    euromillioner                      # == Main.main: draws -> 70/30 split -> GBDT x500 -> predict -> check
    euromillioner run [flags]          # same, with flags (reference defaults)
    euromillioner train --model mlp    # 62->128->62 MLP on the fused HIP path (DP via torchrun)
    euromillioner train --model mlp-wide | rf | gbdt
    euromillioner predict --ckpt model.zip [--data-source csv --data-path draws.csv]
    euromillioner gen --n 1000000 --planted 0.9 --out draws.csv
    euromillioner info                 # device, native libraries, kernel inventory

Exit codes: 0 ok, 2 usage/config error, 3 data error, 4 training/runtime error
(the reference always exits 0 and reports every failure as "Could not access URL",
``Main.java:144-147``, defect D-g).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import traceback

from . import config as C
from . import log as L

# flag -> dotted config key
_FLAGS = {
    "--data-source": "data.source", "--data-path": "data.path", "--from-date": "data.from_date",
    "--to-date": "data.to_date", "--html-table-class": "data.html_table_class", "--train-pct": "data.train_pct",
    "--date-format": "data.date_format", "--label-column": "data.label_column", "--n-draws": "data.n_draws",
    "--seed": "data.seed", "--planted": "data.planted", "--lags": "data.lags", "--workdir": "data.workdir",
    "--header": "data.header", "--fetch-jitter-ms": "data.fetch_jitter_ms", "--device-gb": "data.device_gb",
    "--eta": "gbdt.eta", "--max-depth": "gbdt.max_depth", "--objective": "gbdt.objective",
    "--subsample": "gbdt.subsample", "--nthread": "gbdt.nthread", "--gamma": "gbdt.gamma",
    "--eval-metric": "gbdt.eval_metric", "--nround": "gbdt.nround", "--lambda": "gbdt.reg_lambda",
    "--min-child-weight": "gbdt.min_child_weight", "--num-class": "gbdt.num_class", "--target": "gbdt.target", "--max-bin": "gbdt.max_bin",
    "--trees": "rf.n_trees", "--rf-max-depth": "rf.max_depth", "--min-samples-leaf": "rf.min_samples_leaf",
    "--feature-subset": "rf.feature_subset",
    "--hidden": "mlp.hidden", "--activation": "mlp.activation", "--loss": "mlp.loss", "--lr": "mlp.lr",
    "--batch": "mlp.batch", "--accum": "mlp.accum", "--steps": "mlp.steps", "--epochs": "mlp.epochs", "--dtype": "mlp.dtype",
    "--weight-decay": "mlp.weight_decay", "--eval-every": "mlp.eval_every",
    "--dp": "dist.dp", "--backend": "dist.backend", "--bucket-mb": "dist.bucket_mb", "--timeout": "dist.timeout_s",
    "--comm-dtype": "dist.comm_dtype",
    "--fault-at-step": "dist.fault_at_step", "--fault-rank": "dist.fault_rank",
    "--check-sync-every": "dist.check_sync_every", "--avg-frequency": "dist.avg_frequency",
    "--max-restarts": "dist.max_restarts",
    "--profile-dir": "log.profile_dir", "--profile-steps": "log.profile_steps",
    "--ckpt": "ckpt.path", "--resume": "ckpt.resume", "--ckpt-every": "ckpt.every",
    "--log-level": "log.level", "--device": "device",
}


def _add_common(p: argparse.ArgumentParser):
    p.add_argument("--config", default=None, help="YAML/JSON config file")
    for flag, key in _FLAGS.items():
        p.add_argument(flag, dest=key.replace(".", "__"), default=None)
    p.add_argument("--reference-compat", action="store_true",
                   help="train a 2nd booster on the validation split and compare (Main.java:138)")


def _cfg_from_args(a, extra: dict | None = None) -> C.RunConfig:
    over = {}
    for flag, key in _FLAGS.items():
        v = getattr(a, key.replace(".", "__"), None)
        if v is not None:
            over[key] = v
    over.update(extra or {})
    cfg = C.build_config(a.config, over)
    if getattr(a, "reference_compat", False):
        cfg.reference_compat = True
    return cfg


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="euromillioner", description=__doc__.split("\n\n")[0])
    sub = ap.add_subparsers(dest="cmd")
    p = sub.add_parser("run", help="reference pipeline (default)")
    _add_common(p)
    p = sub.add_parser("train", help="train a model (mlp | mlp-wide | rf | gbdt)")
    _add_common(p)
    p.add_argument("--model", default="mlp", choices=["mlp", "mlp-wide", "rf", "gbdt"])
    p = sub.add_parser("predict", help="predict the next draw from a checkpoint")
    _add_common(p)
    p.add_argument("--model", default=None, choices=["mlp", "mlp-wide", "rf", "gbdt"])
    p = sub.add_parser("gen", help="write synthetic draws to CSV")
    p.add_argument("--n", "--n-draws", dest="n", type=int, default=None, help="draws to generate (same name as train --n-draws)")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--planted", type=float, default=0.0)
    p.add_argument("--out", required=True)
    p.add_argument("--format", default="csv", choices=["csv", "reference", "html"])
    sub.add_parser("info", help="environment / native library report")
    return ap


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = build_parser()
    if not argv or argv[0].startswith("-") and argv[0] not in ("-h", "--help"):
        argv = ["run"] + argv  # no subcommand == Main.main
    try:
        a = ap.parse_args(argv)
    except SystemExit as e:
        return int(e.code or 0) if e.code in (0, None) else 2
    if a.cmd == "info":
        return _info()
    if a.cmd == "gen":
        return _gen(a)
    try:
        cfg = _cfg_from_args(a, {"model": a.model} if getattr(a, "model", None) else None)
    except (KeyError, ValueError) as e:
        L.setup("INFO")
        L.get("Main").error(f"invalid configuration: {e}")
        return 2
    L.setup(cfg.log.level, rank=int(os.environ.get("RANK", "0")) if "RANK" in os.environ else None)
    log = L.get("Main")
    if a.cmd in ("run", "train"):
        # --dp N: N ranks on this node.  Under torchrun (WORLD_SIZE set) it must match the launch;
        # otherwise this process starts the N ranks itself (parallel/launch.py) and waits.
        from .parallel import launch

        try:
            world, must_spawn = launch.requested_world(cfg.dist.dp)
        except ValueError as e:
            log.error(f"invalid configuration: {e}")
            return 2
        if must_spawn:
            log.info(f"launching {world} ranks (127.0.0.1 rendezvous)"
                     + (f", up to {cfg.dist.max_restarts} restart(s)" if cfg.dist.max_restarts else ""))
            base = [sys.executable, "-m", "euromillioner_amd"] + argv
            # a restarted job continues from the last checkpoint (ckpt.path) when there is one
            again = base + ["--resume", "auto"] if cfg.ckpt.path and not cfg.ckpt.resume else base
            return launch.spawn(base, world, timeout_s=float(os.environ.get("EUROM_LAUNCH_TIMEOUT", "86400")),
                                max_restarts=int(cfg.dist.max_restarts), restart_argv=again)
    try:
        if a.cmd == "run":
            from .pipeline import run_reference_pipeline

            res = run_reference_pipeline(cfg)
        elif a.cmd == "train":
            from .train import train

            res = train(cfg)
        elif a.cmd == "predict":
            from .train import predict_next

            res = predict_next(cfg)
        else:
            ap.print_help()
            return 2
    except (FileNotFoundError, ValueError) as e:
        log.error(f"data/config error: {e}")
        log.debug(traceback.format_exc())
        return 3
    except Exception as e:  # noqa: BLE001
        log.error(f"{type(e).__name__}: {e}")
        log.debug(traceback.format_exc())
        return 4
    if res is not None and (int(os.environ.get("RANK", "0")) == 0) and cfg.log.json_metrics:
        L.metrics_line(res)
    return 0


def _gen(a) -> int:
    from .data.draws import DrawSet

    ds = DrawSet.synthetic(n=a.n, seed=a.seed, planted=a.planted)
    if a.format == "csv":
        from .data.csv_io import write_draws_csv

        write_draws_csv(a.out, ds)
    elif a.format == "reference":
        from .data.csv_io import write_reference_csv

        base = a.out[:-4] if a.out.endswith(".csv") else a.out
        write_reference_csv(base + ".csv", base + "_validation.csv", ds)
    else:
        from .data.html_table import render_results_table

        with open(a.out, "w", encoding="utf-8") as f:
            f.write(render_results_table(ds))
    print(json.dumps({"written": a.out, "draws": len(ds)}))
    return 0


def _info() -> int:
    import platform

    info = {"python": platform.python_version()}
    try:
        import torch

        info["torch"] = torch.__version__
        info["hip"] = torch.version.hip
        info["gpu"] = torch.cuda.is_available()
        if info["gpu"]:
            p = torch.cuda.get_device_properties(0)
            info["device"] = {"name": p.name, "cus": p.multi_processor_count, "mem_gb": round(p.total_memory / 2**30)}
            info["device_count"] = torch.cuda.device_count()
        import torch.distributed as dist

        info["rccl"] = dist.is_nccl_available()
    except Exception as e:  # noqa: BLE001
        info["torch_error"] = str(e)
    from . import _build

    info["native"] = {"hip_lib": os.path.exists(_build.lib_path()), "host_lib": os.path.exists(_build.host_lib_path())}
    print(json.dumps(info))
    return 0


if __name__ == "__main__":
    sys.exit(main())
