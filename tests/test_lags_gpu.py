"""Lag windows on the GPU engines (data.lags > 1): the device lag-window one-hot
(csrc/metrics.hip onehot_lags) vs data.draws.lag_features, and GemmMLPTrainer(lags=k) gradients vs a
plain PyTorch fp32 DrawMLP on the same windows; checkpoints round-trip the [N, 62k] layer-0 weight."""
import numpy as np
import pytest
import torch

from euromillioner_amd.data.draws import DrawSet, lag_features

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-12))


@pytest.mark.parametrize("lags,dtype", [(1, torch.bfloat16), (3, torch.bfloat16), (4, torch.float32)])
def test_onehot_lags_matches_lag_features(lags, dtype):
    from euromillioner_amd.ops import fused_mlp as FM

    ds = DrawSet.synthetic(n=700, seed=2, planted=0.5, calendar=False)
    masks = FM.rows_to_masks(torch.from_numpy(ds.numbers).cuda())
    X, _ = lag_features(ds.numbers, lags)
    B, off = 300, 17
    got = FM.onehot_lags(masks, B, lags, offset=off, dtype=dtype).float().cpu().numpy().reshape(B, lags, 64)
    assert (got[:, :, 62:] == 0).all()
    assert np.array_equal(got[:, :, :62].reshape(B, 62 * lags), X[off:off + B])
    sidx = torch.tensor([5, 0, 99, 3], dtype=torch.int32, device="cuda")
    g2 = FM.onehot_lags(masks, 4, lags, sidx=sidx, dtype=dtype).float().cpu().numpy().reshape(4, lags, 64)
    assert np.array_equal(g2[:, :, :62].reshape(4, 62 * lags), X[[5, 0, 99, 3]])


@pytest.mark.parametrize("dtype,tol", [("fp32", 1e-4), ("bf16", 3e-2)])
def test_lag_trainer_grads_match_torch(dtype, tol):
    from euromillioner_amd.models.gemm_mlp import GemmMLPTrainer
    from euromillioner_amd.models.mlp import DrawMLP
    from euromillioner_amd.ops.fused_mlp import rows_to_masks

    lags = 3
    ds = DrawSet.synthetic(n=5000, seed=4, planted=0.6, calendar=False)
    masks = rows_to_masks(torch.from_numpy(ds.numbers).cuda())
    sizes, B, off = (62 * lags, 128, 62), 2048, 11
    tr = GemmMLPTrainer(sizes, seed=5, dtype=dtype, lags=lags)
    ref = DrawMLP(sizes, seed=5)
    X, Y = lag_features(ds.numbers, lags)
    xb, yb = torch.from_numpy(X[off:off + B]), torch.from_numpy(Y[off:off + B])
    loss = ref.loss(ref(xb), yb)
    loss.backward()
    lk, gk = tr.grads_only(masks, B, offset=off)
    assert abs(lk - loss.item()) < (1e-5 if dtype == "fp32" else 1e-2) * max(1, loss.item())
    for n, p in ref.named_parameters():
        assert gk[n].shape == p.grad.shape, n
        assert _rel(gk[n], p.grad) < tol, n
    sd = tr.state_dict()  # logical [N, 62k] weights round-trip through the padded layout
    for n, p in ref.state_dict().items():
        assert torch.equal(sd[n], p), n


def test_lag_cli_trains_on_gemm_engine(tmp_path):
    from euromillioner_amd import config as C
    from euromillioner_amd.ckpt import modelserializer as MS
    from euromillioner_amd.train import train

    ck = str(tmp_path / "lags.zip")
    cfg = C.build_config(None, {"model": "mlp", "device": "cuda", "data.lags": 3, "data.n_draws": 6001,
                                "data.planted": 0.8, "mlp.steps": 100, "mlp.batch": 1024, "mlp.lr": 0.005,
                                "mlp.eval_every": 0, "log.level": "WARN", "ckpt.path": ck}, environ={})
    res = train(cfg)
    assert res["engine"] == "gemm" and res["sizes"] == [186, 128, 62]
    assert res["val"]["acc"] > res["val"]["trivial_acc"], res["val"]
    assert MS.load(ck)["sizes"] == [186, 128, 62]
