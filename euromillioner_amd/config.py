"""Typed configuration.  Every default is the reference's hard-coded constant.

The reference has no config system: ``Main.main`` ignores ``args`` (``Main.java:35``)
and hard-codes every value.  Those literals become defaults here:

==========================  ==================================  ==========================
field                       value                               reference
==========================  ==================================  ==========================
data.from_date/to_date      1900-01-01 .. 2020-06-14            Main.java:37 (URL query)
data.html_table_class       "table table-bordered ..."          Main.java:62
data.train_pct              70                                  Main.java:83
data.date_format            "E, MMM d, yyyy"                    Main.java:92
data.label_column           0                                   Main.java:110-111
gbdt.*                      gbtree, eta 1.0, max_depth 3,       Main.java:113-126
                            cpu_predictor, reg:logistic,
                            subsample 1, nthread 6, gamma 1.0,
                            eval_metric logloss
gbdt.nround                 500                                 Main.java:136
log.level                   INFO                                log4j.properties:2
==========================  ==================================  ==========================

Precedence (lowest -> highest): dataclass defaults < YAML/JSON file < ``EUROM_*``
environment variables (``EUROM_GBDT__ETA=0.3``) < explicit CLI flags.
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Any

REFERENCE_URL = ("http://portalseven.com/lottery/euromillions_winning_numbers.jsp"
                 "?fromDate=1900-01-01&toDate=2020-06-14&viewType=3")  # Main.java:37 (never fetched here)
REFERENCE_TABLE_CLASS = "table table-bordered table-condensed table-striped text-center table-hover"  # Main.java:62


@dataclasses.dataclass
class DataConfig:
    source: str = "synthetic"  # synthetic | csv | html | reference-csv | device (generated on the GPU)
    path: str | None = None
    from_date: str = "1900-01-01"
    to_date: str = "2020-06-14"
    html_table_class: str = REFERENCE_TABLE_CLASS
    train_pct: float = 70.0
    date_format: str = "E, MMM d, yyyy"
    label_column: int = 0
    n_draws: int | None = None  # synthetic: None = the reference's calendar range (~1.33k draws)
    seed: int = 0
    planted: float = 0.0  # synthetic Markov structure strength (0 = iid draws)
    lags: int = 1
    workdir: str | None = None  # where the emn*.csv split files go (None: a temp dir, removed afterwards; D-h)
    header: str = "auto"  # CSV header handling: auto | yes | no (D-b / D-c)
    fetch_jitter_ms: int = 0  # Main.java:53-54 random pre-fetch sleep; accepted for parity, no network here
    device_gb: float = 0.0  # source=device: GiB of HBM-resident draw masks (8 B each) unless n_draws is set


@dataclasses.dataclass
class GBDTConfig:
    booster: str = "gbtree"
    eta: float = 1.0
    max_depth: int = 3
    predictor: str = "cpu_predictor"  # accepted for parity; prediction runs on the GPU kernel when available
    objective: str = "reg:logistic"
    subsample: float = 1.0
    silent: int = 1  # deprecated XGBoost key kept for parity (defect D-j)
    nthread: int = 6
    gamma: float = 1.0
    eval_metric: str = "logloss"
    nround: int = 500
    reg_lambda: float = 1.0  # XGBoost default
    min_child_weight: float = 1.0  # XGBoost default
    base_score: float = 0.5  # XGBoost default
    max_bin: int = 256
    num_class: int = 0  # multi:softprob / multi:softmax (0 = max label + 1)
    target: str = "next-draw"  # next-draw (62 boosters) | reference (label_column of the raw features; D-d)
    device: str = "auto"  # auto | cuda | cpu


@dataclasses.dataclass
class RFConfig:
    n_trees: int = 100
    max_depth: int = 8
    min_samples_leaf: int = 1
    feature_subset: str = "sqrt"  # sqrt | all | log2 | <float fraction>
    bootstrap: bool = True
    seed: int = 0
    device: str = "auto"


@dataclasses.dataclass
class MLPConfig:
    model: str = "mlp"  # mlp (62-128-62 fused) | mlp-wide (62-8192-8192-62) | custom
    hidden: tuple = (128,)
    activation: str = "relu"
    loss: str = "softmax"  # softmax (grouped 50/12 CE) | bce
    lr: float = 3e-3
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.0
    batch: int = 1 << 20
    accum: int = 1  # GEMM engine: micro-batches per optimizer step (gradient accumulation; batch % accum == 0)
    steps: int = 200
    epochs: int | None = None
    dtype: str = "bf16"
    seed: int = 0
    eval_every: int = 50
    shuffle: bool = True


@dataclasses.dataclass
class DistConfig:
    dp: int = 1  # ranks on this node: > 1 without a torchrun env -> the CLI launches them (parallel/launch.py)
    backend: str = "auto"  # auto -> nccl (RCCL) on GPU, gloo on CPU
    bucket_mb: float = 25.0
    comm_dtype: str = "fp32"  # GEMM engine gradient wire: fp32, or bf16 (half the all-reduce bytes)
    timeout_s: float = 300.0
    fault_at_step: int | None = None  # test-only fault injection
    fault_rank: int | None = None
    check_sync_every: int = 0  # cross-rank parameter checksum assert every k steps (0 = off)
    avg_frequency: int = 0  # >0: parameter averaging every k local steps (Spark ParameterAveraging parity)
    max_restarts: int = 0  # self-launched --dp N jobs: restart every rank (with --resume auto) after a failure


@dataclasses.dataclass
class CkptConfig:
    path: str | None = None
    resume: str | None = None  # a checkpoint path, or "auto" = ckpt.path if it exists (restart-safe)
    every: int = 0


@dataclasses.dataclass
class LogConfig:
    level: str = "INFO"
    json_metrics: bool = True
    profile_dir: str | None = None  # torch.profiler chrome trace of a few training steps
    profile_steps: int = 5


@dataclasses.dataclass
class RunConfig:
    data: DataConfig = dataclasses.field(default_factory=DataConfig)
    gbdt: GBDTConfig = dataclasses.field(default_factory=GBDTConfig)
    rf: RFConfig = dataclasses.field(default_factory=RFConfig)
    mlp: MLPConfig = dataclasses.field(default_factory=MLPConfig)
    dist: DistConfig = dataclasses.field(default_factory=DistConfig)
    ckpt: CkptConfig = dataclasses.field(default_factory=CkptConfig)
    log: LogConfig = dataclasses.field(default_factory=LogConfig)
    model: str = "gbdt"  # gbdt | rf | mlp | mlp-wide
    device: str = "auto"
    reference_compat: bool = False  # reproduce D-f (second booster trained on validation) + checkPredicts

    # ------------------------------------------------------------------ helpers
    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    def gbdt_params(self) -> dict:
        """The reference's XGBoost parameter map (Main.java:113-126)."""
        g = self.gbdt
        p = {"booster": g.booster, "eta": g.eta, "max_depth": g.max_depth, "predictor": g.predictor,
             "objective": g.objective, "subsample": g.subsample, "silent": g.silent, "nthread": g.nthread,
             "gamma": g.gamma, "eval_metric": g.eval_metric}
        if g.objective.startswith("multi:"):
            p["num_class"] = g.num_class
        return p


def _coerce(cur: Any, val: Any, typ: Any = None):
    if isinstance(val, str):
        if isinstance(cur, bool) or typ in (bool, "bool"):
            return val.strip().lower() in ("1", "true", "yes", "on")
        if isinstance(cur, int) and not isinstance(cur, bool):
            return int(val)
        if isinstance(cur, float):
            return float(val)
        if isinstance(cur, tuple):
            parts = [p for p in val.replace("x", ",").split(",") if p.strip()]
            return tuple(type(cur[0])(p) if cur else float(p) for p in parts)
        if cur is None:
            low = val.strip().lower()
            if low in ("none", "null", ""):
                return None
            for conv in (int, float):
                try:
                    return conv(val)
                except ValueError:
                    pass
        return val
    if isinstance(cur, tuple) and isinstance(val, list):
        return tuple(val)
    return val


def set_path(cfg: RunConfig, dotted: str, value: Any) -> None:
    obj: Any = cfg
    parts = dotted.split(".")
    for p in parts[:-1]:
        obj = getattr(obj, p)
    leaf = parts[-1]
    if not hasattr(obj, leaf):
        raise KeyError(f"unknown config key {dotted}")
    setattr(obj, leaf, _coerce(getattr(obj, leaf), value))


def apply_mapping(cfg: RunConfig, mapping: dict, prefix: str = "") -> None:
    for k, v in mapping.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            apply_mapping(cfg, v, key + ".")
        else:
            set_path(cfg, key, v)


def load_file(cfg: RunConfig, path: str) -> None:
    with open(path, encoding="utf-8") as f:
        text = f.read()
    if path.endswith((".yaml", ".yml")):
        import yaml

        data = yaml.safe_load(text) or {}
    else:
        data = json.loads(text)
    apply_mapping(cfg, data)


def apply_env(cfg: RunConfig, environ=None) -> None:
    """EUROM_<SECTION>__<FIELD>=value  (e.g. EUROM_GBDT__ETA=0.3, EUROM_MODEL=rf)."""
    env = os.environ if environ is None else environ
    for k, v in env.items():
        if not k.startswith("EUROM_") or k in ("EUROM_AUTOBUILD", "EUROM_FORCE_BUILD", "EUROM_OFFLOAD_ARCH"):
            continue
        dotted = k[len("EUROM_"):].lower().replace("__", ".")
        try:
            set_path(cfg, dotted, v)
        except (KeyError, AttributeError):
            continue


# enumerated fields: a typo must be a configuration error (exit 2), not a silently ignored value
CHOICES = {
    "model": ("gbdt", "rf", "mlp", "mlp-wide"),
    "device": ("auto", "cuda", "cpu"),
    "data.source": ("synthetic", "csv", "html", "reference-csv", "device"),
    "gbdt.objective": ("reg:logistic", "binary:logistic", "reg:squarederror", "multi:softprob", "multi:softmax"),
    "gbdt.eval_metric": ("logloss", "rmse", "error", "mlogloss", "merror"),
    "gbdt.device": ("auto", "cuda", "cpu"),
    "rf.device": ("auto", "cuda", "cpu"),
    "mlp.activation": ("relu", "sigmoid", "tanh"),
    "mlp.loss": ("softmax", "bce"),
    "mlp.dtype": ("bf16", "fp32"),
    "dist.backend": ("auto", "nccl", "gloo"),
}


def validate(cfg: RunConfig) -> RunConfig:
    for dotted, allowed in CHOICES.items():
        obj: Any = cfg
        for part in dotted.split("."):
            obj = getattr(obj, part)
        if obj not in allowed:
            raise ValueError(f"{dotted}={obj!r}: expected one of {', '.join(allowed)}")
    if cfg.mlp.accum < 1 or cfg.mlp.batch % cfg.mlp.accum:
        raise ValueError(f"mlp.accum={cfg.mlp.accum}: must be >= 1 and divide mlp.batch={cfg.mlp.batch}")
    if cfg.dist.comm_dtype not in ("fp32", "bf16"):
        raise ValueError(f"dist.comm_dtype={cfg.dist.comm_dtype!r}: must be fp32 or bf16")
    if cfg.dist.dp < 1 or cfg.dist.dp > 64:
        raise ValueError(f"dist.dp={cfg.dist.dp}: must be in 1..64 (ranks of one node)")
    if cfg.data.source == "device" and not cfg.data.n_draws and cfg.data.device_gb <= 0:
        raise ValueError("data.source=device needs data.n_draws or data.device_gb")
    return cfg


def build_config(file: str | None = None, overrides: dict | None = None, environ=None) -> RunConfig:
    cfg = RunConfig()
    if file:
        load_file(cfg, file)
    apply_env(cfg, environ)
    for k, v in (overrides or {}).items():
        if v is not None:
            set_path(cfg, k, v)
    return validate(cfg)
