"""``euromillioner train`` / ``predict`` (T5 trainers, T6 checkpoints, T4 data parallelism).

The reference has exactly one "training" call site — ``XGBoost.train`` x2 in
``Main.java:128-138`` — and no MLP/RF/DP at all; the north star adds them
(``BASELINE.json``).  This module wires the engines to the config/CLI:

===========  ==============================================  =============================
model        engine (first that applies)                     distributed
===========  ==============================================  =============================
mlp          fused single-launch HIP kernel (62->128->62)     grad all-reduce (C1), RCCL
             -> GEMM trainer (other sizes, GPU)              per-layer async buckets (C1)
             -> DrawMLP + torch Adam (CPU / lags > 1)        GradBucketer hooks (C1), gloo
mlp-wide     GEMM trainer, 62->8192->8192->62                per-layer async buckets (C1)
rf           HIP forest engine / numpy oracle                tree-parallel + all-gather (C5)
gbdt         reference pipeline (XGBoost semantics)          single process
===========  ==============================================  =============================

Data parallelism is one process per device (``torchrun``); every rank reads the same
draw sequence and trains on its contiguous shard of the training split; the global
batch ``mlp.batch`` is split evenly across ranks.  MLP checkpoints are DL4J
``ModelSerializer``-layout zips (:mod:`euromillioner_amd.ckpt.modelserializer`)
carrying the Adam state, so ``--resume`` continues exactly.
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch

from . import log as L
from .ckpt import modelserializer as MS
from .config import RunConfig
from .data.draws import lag_features, multi_hot, positional_split
from .parallel import dist as D
from .pipeline import date_str, load_draws, next_draw_date, run_reference_pipeline


# ---------------------------------------------------------------------------------------------
# engines: one interface over the three MLP implementations
# ---------------------------------------------------------------------------------------------
class _Engine:
    name = "base"

    def step(self, idx: torch.Tensor | None, offset: int, B: int, global_batch: int) -> torch.Tensor:
        raise NotImplementedError

    def evaluate(self, offset: int, n: int) -> dict:
        raise NotImplementedError

    n_local = 0  # local steps taken (parameter-averaging phase; restored on resume)
    avg_k = 0

    def finish(self) -> None:
        """End of training: with --avg-frequency k, average once more unless the last local step
        just did (Spark's ParameterAveragingTrainingMaster averages at the end of every fit), so the
        final evaluation, the checkpoint and the cross-rank check see one model."""
        if self.avg_k > 0 and self.n_local % self.avg_k != 0:
            self.average_parameters()
            self.n_local = 0

    def average_parameters(self) -> None:
        pass


def _checksum(flat: torch.Tensor) -> torch.Tensor:
    """Order-sensitive integer checksum of a float buffer (bit-exact comparison across ranks)."""
    bits = flat.detach().reshape(-1).view(torch.int32).to(torch.int64)
    w = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 65521 + 1
    return torch.stack([bits.sum(), (bits * w).sum()])


def check_sync(engine: "_Engine", info: D.DistInfo) -> None:
    """Race/desync detector: every rank must hold bit-identical parameters."""
    if not info.is_dist:
        return
    c = _checksum(engine.flat_params())
    if info.backend == "gloo":
        c = c.cpu()
    allc = [torch.zeros_like(c) for _ in range(info.world)]
    torch.distributed.all_gather(allc, c)
    if any(not torch.equal(allc[0], x) for x in allc[1:]):
        raise RuntimeError("data-parallel ranks diverged: parameter checksums differ " +
                           str([x.tolist() for x in allc]))


def _sharded_eval(model, masks, offset: int, n: int) -> dict:
    """C3: each rank scores its slice of the validation range; the model all-reduces the sums."""
    if model.group is None:
        return model.evaluate(masks, n, offset=offset)
    import torch.distributed as dist

    a, b = D.shard_range(n, D.DistInfo(dist.get_rank(model.group), dist.get_world_size(model.group)))
    return model.evaluate(masks, b - a, offset=offset + a)


class _FusedEngine(_Engine):
    """62->128->62 on csrc/mlp_fused.hip + csrc/adam.hip."""

    name = "fused"
    _MAP = {"layers.0.weight": "l1.weight", "layers.0.bias": "l1.bias", "layers.1.weight": "l2.weight",
            "layers.1.bias": "l2.bias"}

    def __init__(self, cfg: RunConfig, info: D.DistInfo, masks: torch.Tensor, sd: dict):
        from .models.mlp import FusedSmallMLP

        m = cfg.mlp
        self.model = FusedSmallMLP(info.device, loss=m.loss, lr=m.lr, betas=tuple(m.betas), eps=m.eps,
                                   weight_decay=m.weight_decay, state_dict={self._MAP[k]: v for k, v in sd.items()},
                                   process_group=info.group, dtype=m.dtype)
        self.masks = masks

    def step(self, idx, offset, B, global_batch):
        return self.model.step(self.masks, B, offset=offset, sidx=idx, global_batch=global_batch)

    def evaluate(self, offset, n):
        return _sharded_eval(self.model, self.masks, offset, n)

    def state_dict(self):
        inv = {v: k for k, v in self._MAP.items()}
        return {inv[k]: v for k, v in self.model.state_dict().items()}

    def optimizer_state(self):
        st = self.model.optimizer_state()
        inv = {v: k for k, v in self._MAP.items()}
        return {"m": {inv[k]: v for k, v in st["m"].items()}, "v": {inv[k]: v for k, v in st["v"].items()},
                "step": st["step"]}

    def load_optimizer_state(self, st):
        self.model.load_optimizer_state({"m": {self._MAP[k]: v for k, v in st["m"].items()},
                                         "v": {self._MAP[k]: v for k, v in st["v"].items()}, "step": st["step"]})

    def broadcast(self):
        self.model.broadcast_parameters()

    def flat_params(self):
        return self.model.params


class _GemmEngine(_Engine):
    """Any 62->...->62 stack on the K1-K3 GEMMs + K10 loss + flat Adam."""

    name = "gemm"

    def __init__(self, cfg: RunConfig, info: D.DistInfo, masks: torch.Tensor, sizes, sd: dict):
        from .models.gemm_mlp import GemmMLPTrainer

        m = cfg.mlp
        self.info = info
        # --avg-frequency k (Spark ParameterAveraging parity): local steps, flat parameter + moment
        # averaging every k steps; otherwise synchronous gradient all-reduce inside the step
        self.avg_k = int(cfg.dist.avg_frequency or 0)
        self.model = GemmMLPTrainer(sizes, info.device, activation=m.activation, loss=m.loss, lr=m.lr,
                                    betas=tuple(m.betas), eps=m.eps, weight_decay=m.weight_decay, state_dict=sd,
                                    process_group=None if self.avg_k > 0 else info.group,
                                    bucket_mb=cfg.dist.bucket_mb, dtype=m.dtype, lags=cfg.data.lags,
                                    comm_dtype=cfg.dist.comm_dtype)
        self.masks = masks
        self.accum = m.accum
        self.n_local = 0

    def step(self, idx, offset, B, global_batch):
        k = self.accum
        gb = B if self.avg_k > 0 else global_batch  # local steps average over the local batch
        if k > 1:  # B consecutive samples as k micro-batches (gradient accumulation)
            out = self.model.step(self.masks, B // k, offset=offset, global_batch=gb, accum=k)
        else:
            out = self.model.step(self.masks, B, offset=offset, sidx=idx, global_batch=gb)
        if self.avg_k > 0:
            self.n_local += 1
            if self.n_local % self.avg_k == 0 and self.info.is_dist:
                self.model.average_parameters(self.info.group)
            if self.info.is_dist:
                out = out.clone()
                torch.distributed.all_reduce(out)
                out /= self.info.world
        return out

    def evaluate(self, offset, n):
        return _sharded_eval(self.model, self.masks, offset, n)

    def state_dict(self):
        return self.model.state_dict()

    def optimizer_state(self):
        return self.model.optimizer_state()

    def load_optimizer_state(self, st):
        self.model.load_optimizer_state(st)

    def broadcast(self):
        self.model.broadcast_parameters(group=self.info.group)

    def flat_params(self):
        return self.model.params

    def average_parameters(self):
        if self.info.is_dist:
            self.model.average_parameters(self.info.group)


class _TorchEngine(_Engine):
    """CPU plumbing engine (BASELINE.json config 1): DrawMLP in PyTorch + torch.optim.Adam + bucketed
    gradient all-reduce overlapped with backward (GradBucketer).  Every GPU run takes the fused or
    the GEMM engine (HIP kernels end to end, fused Adam), lag windows and parameter averaging
    included."""

    name = "torch"

    def __init__(self, cfg: RunConfig, info: D.DistInfo, X: torch.Tensor, Y: torch.Tensor, sizes, sd: dict):
        from .models.mlp import DrawMLP
        from .parallel.buckets import GradBucketer

        m = cfg.mlp
        self.info = info
        # --dtype fp32 on the GPU: plain fp32 layers (the HIP autograd GEMMs are bf16).  The CPU
        # plumbing path (BASELINE config 1) always computes in fp32.
        self.net = DrawMLP(sizes, activation=m.activation, loss=m.loss,
                           use_hip=False if m.dtype == "fp32" else None).to(info.device)
        self.net.load_state_dict(sd)
        self.opt = torch.optim.Adam(self.net.parameters(), lr=m.lr, betas=tuple(m.betas), eps=m.eps,
                                    weight_decay=m.weight_decay)
        self.bucketer = GradBucketer(self.net, cfg.dist.bucket_mb, group=info.group, world=info.world)
        self.avg_k = int(cfg.dist.avg_frequency or 0)
        if self.avg_k > 0:
            self.bucketer.enabled = False  # local steps; parameters are averaged every avg_k steps
        self.n_local = 0
        self.X, self.Y = X, Y
        self.loss_name = m.loss

    def step(self, idx, offset, B, global_batch):
        if idx is not None:
            x, y = self.X[idx.long()], self.Y[idx.long()]
        else:
            x, y = self.X[offset:offset + B], self.Y[offset:offset + B]
        self.bucketer.zero_grad()
        # local mean * (B * world / global_batch): all-reduce of the mean over ranks == global mean
        loss = self.net.loss(self.net(x), y) * (B * self.info.world / global_batch)
        loss.backward()
        self.bucketer.finish()
        self.opt.step()
        self.n_local += 1
        if self.avg_k > 0 and self.n_local % self.avg_k == 0:
            self.average_parameters()
        out = loss.detach().reshape(1)
        if self.info.is_dist:
            torch.distributed.all_reduce(out)
            out /= self.info.world
        return out

    @torch.no_grad()
    def evaluate(self, offset, n):
        from .models.losses import draw_metrics_torch

        a, b = offset, offset + n
        if self.info.is_dist:  # every rank scores its slice of the validation range
            per = D.shard_range(n, self.info)
            a, b = offset + per[0], offset + per[1]
        z = self.net(self.X[a:b])
        r = draw_metrics_torch(z, self.Y[a:b], self.loss_name) if b > a else None
        keys = ("loss", "acc", "acc_thr", "hits_main", "hits_star", "exact", "trivial_acc")
        vec = torch.tensor([r[k] * (b - a) for k in keys] + [b - a] if r else [0.0] * 7 + [0.0], dtype=torch.float64)
        if self.info.is_dist:
            vec = vec.to(self.info.device) if self.info.backend == "nccl" else vec
            torch.distributed.all_reduce(vec)
            vec = vec.cpu()
        cnt = max(float(vec[7]), 1.0)
        out = {k: float(vec[i]) / cnt for i, k in enumerate(keys)}
        out["count"] = int(vec[7])
        return out

    def state_dict(self):
        return {k: v.detach().float().cpu().clone() for k, v in self.net.state_dict().items()}

    def optimizer_state(self):
        m, v, step = {}, {}, 0
        for name, p in self.net.named_parameters():
            st = self.opt.state.get(p, {})
            m[name] = st.get("exp_avg", torch.zeros_like(p)).detach().float().cpu().clone()
            v[name] = st.get("exp_avg_sq", torch.zeros_like(p)).detach().float().cpu().clone()
            step = int(float(st.get("step", 0)))
        return {"m": m, "v": v, "step": step}

    def load_optimizer_state(self, st):
        for name, p in self.net.named_parameters():
            self.opt.state[p] = {"step": torch.tensor(float(st["step"])),
                                 "exp_avg": st["m"][name].to(p.device, p.dtype).clone(),
                                 "exp_avg_sq": st["v"][name].to(p.device, p.dtype).clone()}

    def broadcast(self):
        D.broadcast_module_(self.net, self.info)

    def flat_params(self):
        return torch.cat([p.detach().reshape(-1).float() for p in self.net.parameters()])

    def average_parameters(self):
        """Spark ParameterAveragingTrainingMaster parity: mean of params and Adam moments."""
        if not self.info.is_dist:
            return
        with torch.no_grad():
            for p in self.net.parameters():
                torch.distributed.all_reduce(p.data)
                p.data /= self.info.world
                st = self.opt.state.get(p, {})
                for k in ("exp_avg", "exp_avg_sq"):
                    if k in st:
                        torch.distributed.all_reduce(st[k])
                        st[k] /= self.info.world


# ---------------------------------------------------------------------------------------------
# checkpoints (DL4J ModelSerializer layout)
# ---------------------------------------------------------------------------------------------
def _layer_names(n_layers: int):
    return [(f"layers.{i}.weight", f"layers.{i}.bias") for i in range(n_layers)]


def _flat_from_named(named: dict, n_layers: int) -> np.ndarray:
    layers = [(named[w].numpy().T, named[b].numpy()) for w, b in _layer_names(n_layers)]
    return MS.flatten_params(layers)


def _named_from_flat(flat: np.ndarray, sizes) -> dict:
    out = {}
    for i, (W, b) in enumerate(MS.unflatten_params(np.asarray(flat, np.float32), list(sizes))):
        out[f"layers.{i}.weight"] = torch.from_numpy(np.ascontiguousarray(W.T))
        out[f"layers.{i}.bias"] = torch.from_numpy(np.ascontiguousarray(b))
    return out


def save_mlp_checkpoint(path: str, engine: _Engine, cfg: RunConfig, sizes, step: int, extra: dict | None = None):
    sd = engine.state_dict()
    st = engine.optimizer_state()
    n = len(sizes) - 1
    layers = [(sd[w].numpy().T, sd[b].numpy()) for w, b in _layer_names(n)]
    conf = MS.multilayer_configuration(list(sizes), cfg.mlp.activation, cfg.mlp.loss, cfg.mlp.lr, tuple(cfg.mlp.betas),
                                       cfg.mlp.eps, cfg.mlp.seed)
    meta = {"step": int(step), "adam_step": int(st["step"]), "engine": engine.name, "model": cfg.model,
            "lags": cfg.data.lags, "loss": cfg.mlp.loss, "activation": cfg.mlp.activation, "sizes": list(sizes)}
    meta.update(extra or {})
    tmp = path + ".tmp"
    MS.save(tmp, layers, conf, _flat_from_named(st["m"], n), _flat_from_named(st["v"], n), meta)
    os.replace(tmp, path)  # atomic: a crash never leaves a torn checkpoint


def load_mlp_checkpoint(path: str) -> dict:
    ck = MS.load(path)
    sizes = ck["sizes"]
    out = {"sizes": sizes, "state_dict": _named_from_flat(ck["flat"], sizes), "extra": ck.get("extra", {}),
           "config": ck["config"]}
    if "m" in ck:
        out["opt"] = {"m": _named_from_flat(ck["m"], sizes), "v": _named_from_flat(ck["v"], sizes),
                      "step": int(out["extra"].get("adam_step", out["extra"].get("step", 0)))}
    return out


# ---------------------------------------------------------------------------------------------
# MLP training
# ---------------------------------------------------------------------------------------------
def _export_trace(prof, out_dir: str, rank: int) -> None:
    os.makedirs(out_dir, exist_ok=True)
    prof.export_chrome_trace(os.path.join(out_dir, f"trace_rank{rank}.json"))
    with open(os.path.join(out_dir, f"kernels_rank{rank}.txt"), "w", encoding="utf-8") as f:
        f.write(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=40))


def _mlp_sizes(cfg: RunConfig) -> tuple:
    hidden = tuple(int(h) for h in cfg.mlp.hidden)
    if cfg.model == "mlp-wide" and hidden == (128,):
        hidden = (8192, 8192)
    return (62 * cfg.data.lags,) + hidden + (62,)


def _fused_shape(cfg: RunConfig, sizes) -> bool:
    """The configurations the fused train kernel covers (62 -> 128 -> 62 relu, no parameter averaging);
    every other stack, lag window or averaging run takes the GEMM engine."""
    return tuple(sizes) == (62, 128, 62) and cfg.mlp.activation == "relu" and not cfg.dist.avg_frequency


def _pick_engine(cfg: RunConfig, info: D.DistInfo, sizes) -> str:
    if info.device.type != "cuda":
        return "torch"  # CPU plumbing path
    if _fused_shape(cfg, sizes):
        return "fused"  # the fused train kernel: bf16 (mlp_fused.hip) or exact fp32 (mlp_fused_f32.hip)
    return "gemm"  # any other stack, lag windows, parameter averaging


def train_mlp(cfg: RunConfig) -> dict:
    log = L.get("Trainer")
    # RCCL at high stream priority only for the GEMM engine's bucketed all-reduces (parallel/dist.py)
    gemm_like = not _fused_shape(cfg, _mlp_sizes(cfg))  # the same predicate as _pick_engine
    info = D.init(cfg.dist.backend, cfg.dist.timeout_s, device=cfg.device, high_priority=gemm_like)
    try:
        return _train_mlp(cfg, info, log)
    finally:
        D.shutdown(info)


def _train_mlp(cfg: RunConfig, info: D.DistInfo, log) -> dict:
    m = cfg.mlp
    sizes = _mlp_sizes(cfg)
    lags = cfg.data.lags
    device_data = cfg.data.source == "device"
    if device_data:  # HBM-resident draws generated on the GPU (csrc/datagen.hip); no host copy
        from .data.device_gen import gb_to_draws, generate_masks

        if info.device.type != "cuda":
            raise ValueError("data.source=device needs a GPU")
        n_draws = int(cfg.data.n_draws) if cfg.data.n_draws else gb_to_draws(cfg.data.device_gb)
        dmasks = generate_masks(n_draws, seed=cfg.data.seed, planted=cfg.data.planted, device=info.device)
        ds = None
        n_samples = n_draws - lags
    else:
        ds = load_draws(cfg)
        n_samples = len(ds) - lags
    if n_samples < 4:
        raise ValueError(f"need more draws than lags+3 (have {n_samples + lags})")
    margin = positional_split(n_samples, cfg.data.train_pct)
    a, b = D.shard_range(margin, info)
    shard = b - a
    if shard < 1:
        raise ValueError("training split smaller than the number of ranks")
    local_b = max(1, min(shard, math.ceil(m.batch / info.world)))
    if m.accum > 1:
        local_b = max(m.accum, local_b // m.accum * m.accum)
    global_b = local_b * info.world
    steps = m.steps if m.epochs is None else int(m.epochs) * math.ceil(shard / local_b)

    resume_path = cfg.ckpt.resume
    if resume_path == "auto":  # restart-safe (torchrun --max-restarts): continue from ckpt.path if present
        resume_path = cfg.ckpt.path if cfg.ckpt.path and os.path.exists(cfg.ckpt.path) else None
    resume = load_mlp_checkpoint(resume_path) if resume_path else None
    if resume is not None:
        if tuple(resume["sizes"]) != tuple(sizes):
            raise ValueError(f"checkpoint sizes {resume['sizes']} != configured {list(sizes)}")
        sd = resume["state_dict"]
    else:
        from .models.mlp import DrawMLP

        sd = DrawMLP(sizes, activation=m.activation, loss=m.loss, seed=m.seed).state_dict()
    kind = _pick_engine(cfg, info, sizes)
    if device_data and kind == "torch":
        raise ValueError("data.source=device feeds the GPU engines")
    if m.accum > 1 and kind != "gemm":
        raise ValueError(f"mlp.accum applies to the GEMM engine (this run uses {kind}); the fused kernel takes "
                         "any batch in one launch")
    dev = info.device
    if kind in ("fused", "gemm"):
        from .models.mlp import FusedSmallMLP

        masks = dmasks if device_data else FusedSmallMLP.prepare(torch.from_numpy(ds.numbers).to(dev))
        engine = _FusedEngine(cfg, info, masks, sd) if kind == "fused" else _GemmEngine(cfg, info, masks, sizes, sd)
        sample_base = 0  # sample i -> masks[i] -> masks[i+1]
    else:
        X, Y = lag_features(ds.numbers, lags)
        engine = _TorchEngine(cfg, info, torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev), sizes, sd)
        sample_base = 0
    engine.broadcast()  # C2
    start_step = 0
    if resume is not None:
        start_step = int(resume["extra"].get("step", 0))
        if "opt" in resume:
            engine.load_optimizer_state(resume["opt"])
        engine.n_local = start_step  # keeps the --avg-frequency phase of the interrupted run
        log.info(f"resumed from {resume_path} at step {start_step}")
    log.info(f"mlp {'->'.join(map(str, sizes))} engine={engine.name} device={dev} world={info.world} "
             f"train={margin} (shard {shard}) val={n_samples - margin} batch={global_b} steps={steps}")

    # sample-level shuffles need int32 indices and a host permutation of the shard; device datasets
    # (up to HBM size) and gradient accumulation shuffle whole windows of local_b samples instead
    window_shuffle = device_data or m.accum > 1
    use_perm = m.shuffle and local_b < shard and not window_shuffle
    per_epoch = max(1, shard // local_b)
    wperm, wperm_epoch = None, -1
    perm, perm_epoch = None, -1
    ckpt_path = cfg.ckpt.path
    hist = []
    loss_t = None
    prof = None
    if cfg.log.profile_dir:  # step timeline (chrome trace) for the first profile_steps steps
        from torch.profiler import ProfilerActivity, profile

        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if dev.type == "cuda" else [])
        prof = profile(activities=acts, acc_events=True)  # one cycle: keep its events (and no torch warning)
        prof.__enter__()
    t0 = time.time()
    done = 0
    for step in range(start_step, steps):
        D.maybe_inject_fault(step, info, cfg.dist.fault_at_step, cfg.dist.fault_rank)
        if prof is not None and step == start_step + cfg.log.profile_steps:
            prof.__exit__(None, None, None)
            _export_trace(prof, cfg.log.profile_dir, info.rank)
            prof = None
        idx, off = None, a + sample_base
        if use_perm:  # epoch-keyed permutation: a resumed run sees the same sample order
            epoch, k = divmod(step, per_epoch)
            if epoch != perm_epoch:
                g = np.random.default_rng([m.seed, info.rank, epoch])
                perm = torch.from_numpy((a + g.permutation(shard)).astype(np.int32)).to(dev)
                perm_epoch = epoch
            idx = perm[k * local_b:(k + 1) * local_b]
        elif window_shuffle:
            epoch, k = divmod(step, per_epoch)
            if m.shuffle and epoch != wperm_epoch:
                wperm = np.random.default_rng([m.seed, info.rank, epoch]).permutation(per_epoch)
                wperm_epoch = epoch
            off += int(wperm[k] if m.shuffle else k) * local_b
        loss_t = engine.step(idx, off, local_b, global_b)
        done += 1
        last = step == steps - 1
        if last:
            engine.finish()
        if cfg.dist.check_sync_every and (step + 1) % cfg.dist.check_sync_every == 0:
            check_sync(engine, info)
        if (m.eval_every and (step + 1) % m.eval_every == 0) or last:
            n_val = n_samples - margin if not device_data else min(n_samples - margin, 1 << 24)
            ev = engine.evaluate(margin, n_val) if n_samples > margin else {}
            loss = float(loss_t.reshape(-1)[0].item())
            hist.append({"step": step + 1, "loss": loss, **{f"val_{k}": v for k, v in ev.items()}})
            log.info(f"step {step + 1}/{steps} loss {loss:.5f} val_acc {ev.get('acc', float('nan')):.4f} "
                     f"hits {ev.get('hits_main', float('nan')):.3f}+{ev.get('hits_star', float('nan')):.3f}")
        if ckpt_path and cfg.ckpt.every and (step + 1) % cfg.ckpt.every == 0 and not last:
            # --avg-frequency: rank 0's local parameters and moments are not the model every rank
            # resumes from after a restart, so a checkpoint between averaging points averages first
            # (collective; at fixed steps, so a restarted run and an uninterrupted one take the same
            # averages and stay bit-identical).  Limitation: that extra average is part of
            # the trajectory, so with --avg-frequency k a run with --ckpt-every c (c not a multiple of
            # k) differs from the same run without checkpoints; choose c a multiple of k to keep Spark
            # ParameterAveraging's schedule exactly (tests/test_dist.py
            # test_ckpt_at_averaging_points_keeps_trajectory)
            if engine.avg_k > 0 and engine.n_local % engine.avg_k != 0 and info.is_dist:
                engine.average_parameters()
            if info.rank == 0:
                save_mlp_checkpoint(ckpt_path, engine, cfg, sizes, step + 1)
            D.barrier(info)
    if prof is not None:
        prof.__exit__(None, None, None)
        _export_trace(prof, cfg.log.profile_dir, info.rank)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    secs = time.time() - t0
    if cfg.dist.check_sync_every:
        check_sync(engine, info)
    if ckpt_path:
        if info.rank == 0:
            save_mlp_checkpoint(ckpt_path, engine, cfg, sizes, steps)
        D.barrier(info)
    final = hist[-1] if hist else {}
    sps = done * global_b / secs if secs > 0 else None
    return {"val_acc": final.get("val_acc"), "val_logloss": final.get("val_loss"), "samples_per_sec": sps,
            "world_size": info.world, "trivial_acc": final.get("val_trivial_acc"), "model": cfg.model, "engine": engine.name, "sizes": list(sizes), "world": info.world,
            "device": str(dev), "steps": steps, "start_step": start_step, "global_batch": global_b,
            "train_samples": margin, "val_samples": n_samples - margin,
            "seconds": round(secs, 3),
            "loss": final.get("loss"), "val": {k[4:]: v for k, v in final.items() if k.startswith("val_")},
            "history": hist, "checkpoint": ckpt_path}


# ---------------------------------------------------------------------------------------------
# random forest
# ---------------------------------------------------------------------------------------------
def train_rf(cfg: RunConfig) -> dict:
    from .models.forest import RandomForest, draw_features
    from .models.losses import draw_metrics_torch

    log = L.get("Trainer")
    info = D.init(cfg.dist.backend, cfg.dist.timeout_s, device=cfg.rf.device if cfg.rf.device != "auto" else cfg.device)
    try:
        ds = load_draws(cfg)
        X, Y, F = draw_features(ds.numbers, cfg.data.lags)
        n = len(X)
        margin = positional_split(n, cfg.data.train_pct)
        r = cfg.rf
        dev = "cuda" if info.device.type == "cuda" else "cpu"
        t0 = time.time()
        rf = RandomForest(r.n_trees, r.max_depth, r.min_samples_leaf, r.feature_subset, r.bootstrap, r.seed, dev)
        rf.fit(X[:margin], Y[:margin], F, group=info.group)
        secs = time.time() - t0
        log.info(f"forest: {r.n_trees} trees depth {r.max_depth} on {margin} rows ({rf.backend_used}, "
                 f"world {info.world}) in {secs:.3f}s")
        res = {"model": "rf", "backend": rf.backend_used, "world": info.world, "trees": int(len(rf.feat)),
               "train_samples": margin, "val_samples": n - margin, "seconds": round(secs, 3)}
        if n > margin:
            p = rf.predict_proba(X[margin:])
            z = torch.logit(torch.from_numpy(p).double().clamp(1e-7, 1 - 1e-7)).float()
            yt = torch.from_numpy(multi_hot(ds.numbers[margin + cfg.data.lags:]))
            res["val"] = draw_metrics_torch(z, yt[:len(z)], "bce")
        if cfg.ckpt.path and info.rank == 0:
            rf.save(cfg.ckpt.path)
            res["checkpoint"] = cfg.ckpt.path
        return res
    finally:
        D.shutdown(info)


# ---------------------------------------------------------------------------------------------
def train(cfg: RunConfig) -> dict:
    if cfg.model in ("mlp", "mlp-wide"):
        return train_mlp(cfg)
    if cfg.model == "rf":
        return train_rf(cfg)
    if cfg.model == "gbdt":
        return run_reference_pipeline(cfg)
    raise ValueError(f"unknown model {cfg.model!r}")


def _top_pick(p: np.ndarray) -> tuple[list[int], list[int]]:
    main = sorted(int(i) + 1 for i in np.argsort(-p[:50], kind="stable")[:5])
    stars = sorted(int(i) + 1 for i in np.argsort(-p[50:62], kind="stable")[:2])
    return main, stars


def predict_next(cfg: RunConfig) -> dict:
    """Predict the draw after the last one in the configured data from a checkpoint."""
    path = cfg.ckpt.resume or cfg.ckpt.path
    if not path:
        raise ValueError("predict needs --ckpt (or --resume) pointing at a checkpoint")
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    ds = load_draws(cfg)
    if path.endswith(".npz"):
        from .models.forest import RandomForest, draw_features, pack_bits

        rf = RandomForest.load(path)
        lags = rf.F // 62
        x = pack_bits(multi_hot(ds.numbers[len(ds) - lags:]).reshape(1, -1))
        p = rf.predict_proba(x)[0]
        kind = "rf"
    elif path.endswith(".json"):
        from .models.gbdt import GBDT

        g = GBDT.load(path)
        x = multi_hot(ds.numbers[-1:]).astype(np.float64)
        nf = len(g.cuts) if g.cuts is not None else (g.num_feature or 62)
        if nf > 62 and ds.dates is not None:
            from .data.draws import featurize_raw

            x = np.concatenate([x, featurize_raw(ds)[-1:, :4].astype(np.float64)], axis=1)
        p = np.asarray(g.predict(x))[0]
        kind = "gbdt"
    else:
        from .models import losses as LS
        from .models.mlp import DrawMLP

        ck = load_mlp_checkpoint(path)
        sizes = ck["sizes"]
        ex = ck["extra"]
        lags = int(ex.get("lags", sizes[0] // 62))
        net = DrawMLP(sizes, activation=ex.get("activation", "relu"), loss=ex.get("loss", "softmax"), use_hip=False)
        net.load_state_dict(ck["state_dict"])
        x = torch.from_numpy(multi_hot(ds.numbers[len(ds) - lags:]).reshape(1, -1))
        with torch.no_grad():
            z = net(x)[0]
        if ex.get("loss", "softmax") == "softmax":
            p = torch.cat([torch.softmax(z[LS.MAIN], 0), torch.softmax(z[LS.STAR], 0)]).numpy()
        else:
            p = torch.sigmoid(z).numpy()
        kind = "mlp"
    main, stars = _top_pick(np.asarray(p, dtype=np.float64))
    nxt = next_draw_date(ds.dates[-1]) if ds.dates is not None and len(ds.dates) else None
    res = {"model": kind, "checkpoint": path, "after_draw": date_str(ds.dates[-1]) if ds.dates is not None else None,
           "next_draw_date": date_str(nxt) if nxt is not None else None, "main": main, "stars": stars,
           "p_main": [round(float(p[i - 1]), 5) for i in main], "p_stars": [round(float(p[49 + s]), 5) for s in stars]}
    print(" ".join(f"{v:02d}" for v in main) + "  *  " + " ".join(f"{v:02d}" for v in stars))
    return res
