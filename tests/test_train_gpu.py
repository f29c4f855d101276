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


@pytest.mark.parametrize("hidden,lags,engine", [((128,), 1, "fused"), ((256, 128), 1, "gemm"), ((128,), 2, "gemm")])
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


def _nccl_world1():
    import socket

    import torch
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    return dist


@pytest.mark.parametrize("engine", ["fused", "gemm"])
def test_dp_code_path_on_one_rank_matches_local(engine):
    """The RCCL data-parallel step (fused: slab-reduce -> all-reduce -> Adam; GEMM trainer:
    per-layer async bucket all-reduce) on a 1-rank group equals the local step bit for bit."""
    import torch

    from euromillioner_amd.data.draws import DrawSet
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer
    from euromillioner_amd.models.mlp import FusedSmallMLP

    ds = DrawSet.synthetic(n=9000, seed=5, planted=0.7, calendar=False)
    masks = FusedSmallMLP.prepare(torch.from_numpy(ds.numbers).cuda())
    make = (lambda g: FusedSmallMLP("cuda", seed=1, lr=3e-3, process_group=g)) if engine == "fused" else \
        (lambda g: GemmMLPTrainer((62, 256, 256, 62), "cuda", seed=1, lr=3e-3, process_group=g, bucket_mb=0.05))
    local = make(None)
    for k in range(4):
        local.step(masks, 2048, offset=1000 * k)
    dist = _nccl_world1()
    try:
        dp = make(dist.group.WORLD)
        dp.broadcast_parameters()
        for k in range(4):
            loss = dp.step(masks, 2048, offset=1000 * k)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    assert torch.isfinite(loss).all()
    assert torch.allclose(dp.params, local.params, atol=1e-6, rtol=0), float((dp.params - local.params).abs().max())


def test_rccl_step_replays_from_a_hipgraph(monkeypatch):
    """The fused model's RCCL fallback (slab reduce -> RCCL all-reduce -> Adam) replays from a hipGraph
    when opted in (EUROM_RCCL_GRAPH=1; eager by default until a multi-GPU node confirms capture at
    world >= 2): steps captured in one hipGraph and replayed equal the same steps run eagerly, on the
    RCCL model and on a local model."""
    import torch

    monkeypatch.setenv("EUROM_RCCL_GRAPH", "1")

    from euromillioner_amd.data.draws import DrawSet
    from euromillioner_amd.models.mlp import FusedSmallMLP

    ds = DrawSet.synthetic(n=9000, seed=5, planted=0.7, calendar=False)
    masks = FusedSmallMLP.prepare(torch.from_numpy(ds.numbers).cuda())
    dist = _nccl_world1()
    try:
        dp = FusedSmallMLP("cuda", seed=1, lr=3e-3, process_group=dist.group.WORLD, comm="rccl")
        assert dp.comm == "rccl" and dp.graph_safe
        monkeypatch.delenv("EUROM_RCCL_GRAPH")
        assert not dp.graph_safe  # the default: eager RCCL steps
        monkeypatch.setenv("EUROM_RCCL_GRAPH", "1")
        eager = FusedSmallMLP("cuda", seed=1, lr=3e-3, process_group=dist.group.WORLD, comm="rccl")
        for k in (0, 1, 2, 1, 2):  # the same RCCL step, eager, for the graph's equality check below
            eager.step(masks, 2048, offset=1000 * k)
        dp.broadcast_parameters()
        dp.step(masks, 2048, offset=0)  # first step eager (argument checks)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for k in range(1, 3):
                    loss = dp.step(masks, 2048, offset=1000 * k)
        torch.cuda.current_stream().wait_stream(s)
        g.replay()  # steps 1, 2
        torch.cuda.synchronize()
        mid = dp.params.clone()
        g.replay()  # steps 1, 2 again (same offsets) on the updated parameters
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    assert torch.isfinite(loss).all()
    ref = FusedSmallMLP("cuda", seed=1, lr=3e-3)
    for k in (0, 1, 2):
        ref.step(masks, 2048, offset=1000 * k)
    assert torch.allclose(mid, ref.params, atol=1e-6, rtol=0), float((mid - ref.params).abs().max())
    for k in (1, 2):
        ref.step(masks, 2048, offset=1000 * k)
    assert torch.allclose(dp.params, ref.params, atol=1e-6, rtol=0), float((dp.params - ref.params).abs().max())
    assert torch.equal(dp.params, eager.params), float((dp.params - eager.params).abs().max())  # graph == eager
    assert not torch.equal(mid, dp.params)


def test_parameter_averaging_runs_on_the_gemm_engine():
    from euromillioner_amd.train import train

    res = train(_cfg(**{"mlp.steps": 60, "mlp.batch": 1024, "mlp.lr": 0.005, "dist.avg_frequency": 4}))
    assert res["engine"] == "gemm"
    assert res["val"]["acc"] > res["val"]["trivial_acc"], res["val"]


def test_gemm_dp_panels_and_bf16_wire_on_one_rank():
    """The GEMM trainer's panelled wgrad all-reduce (several panels per hidden layer) equals the local
    step bit for bit on a 1-rank RCCL group; the bf16 wire stays within bf16 rounding of it."""
    import torch

    from euromillioner_amd.data.draws import DrawSet
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer
    from euromillioner_amd.models.mlp import FusedSmallMLP

    ds = DrawSet.synthetic(n=9000, seed=6, planted=0.7, calendar=False)
    masks = FusedSmallMLP.prepare(torch.from_numpy(ds.numbers).cuda())
    sizes, B = (62, 512, 512, 62), 1024

    def run(g, wire="fp32"):
        tr = GemmMLPTrainer(sizes, "cuda", seed=2, lr=3e-3, process_group=g, bucket_mb=0.05, comm_dtype=wire)
        tr.panel_ncu = 2  # 512-row layers -> two 256-row wgrad panels
        for k in range(3):
            tr.step(masks, B, offset=1500 * k)
        torch.cuda.synchronize()
        return tr

    local = run(None)
    dist = _nccl_world1()
    try:
        dp = run(dist.group.WORLD)
        assert dp._plan(B)["wgrad"][1] and len(dp.wgrad_panels(1)) == 2
        a, c = dp.offsets[1][0], dp.offsets[1][1]
        assert sum(1 for s0, _ in dp.last_buckets if a <= s0 < c) >= 2
        bf = run(dist.group.WORLD, "bf16")
    finally:
        dist.destroy_process_group()
    assert torch.equal(dp.params, local.params), float((dp.params - local.params).abs().max())
    p0 = GemmMLPTrainer(sizes, "cuda", seed=2).params
    du_local, du_bf = local.params - p0, bf.params - p0
    rel = ((du_bf - du_local).norm() / du_local.norm()).item()
    assert 0 < rel < 0.05, rel  # bf16 gradient rounding through Adam's normalisation, 3 steps
