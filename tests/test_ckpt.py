"""DL4J ModelSerializer-layout checkpoint: byte layout (golden), ordering, roundtrip.

Parity with a real DL4J artifact is unpinned (no JVM / DL4J files offline); the layout
assumptions are the ones documented in euromillioner_amd/ckpt/modelserializer.py.  One of them is
the JSON type-info style of configuration.json: layers, activations, loss functions and the updater
carry Jackson ``@class`` properties (the fully qualified class name).  DL4J 0.9.x may instead have
written some of them as wrapper objects keyed by a short type name; no artifact here decides which,
so the golden tests below pin this builder's own format, not DL4J's."""
import io
import struct
import zipfile

import numpy as np
import torch

from euromillioner_amd.ckpt import modelserializer as MS


def test_nd4j_write_golden_bytes():
    b = MS.nd4j_write(np.array([1.0, -2.0], dtype=np.float32))
    exp = io.BytesIO()
    exp.write(struct.pack(">H", 4) + b"HEAP" + struct.pack(">i", 8) + struct.pack(">H", 3) + b"INT")
    exp.write(struct.pack(">8i", 2, 1, 2, 2, 1, 0, 1, 99))
    exp.write(struct.pack(">H", 4) + b"HEAP" + struct.pack(">i", 2) + struct.pack(">H", 5) + b"FLOAT")
    exp.write(struct.pack(">2f", 1.0, -2.0))
    assert b == exp.getvalue()
    assert np.array_equal(MS.nd4j_read(b), [1.0, -2.0])


def test_flatten_is_fortran_w_then_b():
    W = np.arange(6, dtype=np.float32).reshape(2, 3)  # nIn=2, nOut=3
    b = np.array([10, 11, 12], dtype=np.float32)
    flat = MS.flatten_params([(W, b)])
    assert flat.tolist() == [0, 3, 1, 4, 2, 5, 10, 11, 12]
    (W2, b2), = MS.unflatten_params(flat, [2, 3])
    assert np.array_equal(W2, W) and np.array_equal(b2, b)


def test_save_load_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    sizes = [62, 16, 62]
    layers = [(rng.standard_normal((a, c)).astype(np.float32), rng.standard_normal(c).astype(np.float32))
              for a, c in zip(sizes[:-1], sizes[1:])]
    P = sum(a * c + c for a, c in zip(sizes[:-1], sizes[1:]))
    m, v = rng.standard_normal(P).astype(np.float32), rng.random(P).astype(np.float32)
    conf = MS.multilayer_configuration(sizes, "relu", "softmax", 1e-3)
    p = str(tmp_path / "model.zip")
    MS.save(p, layers, conf, m, v, {"step": 7})
    with zipfile.ZipFile(p) as z:
        assert set(z.namelist()) == {"configuration.json", "coefficients.bin", "updaterState.bin", "euromillioner.json"}
    ck = MS.load(p)
    assert ck["sizes"] == sizes and ck["extra"]["step"] == 7
    for (W, b), (W2, b2) in zip(layers, ck["layers"]):
        assert np.array_equal(W, W2) and np.array_equal(b, b2)
    assert np.array_equal(ck["m"], m) and np.array_equal(ck["v"], v)
    confs = ck["config"]["confs"]
    assert confs[0]["layer"]["@class"].endswith("DenseLayer") and confs[-1]["layer"]["@class"].endswith("OutputLayer")
    assert confs[-1]["layer"]["lossFn"]["@class"].endswith("LossMCXENT")


def test_state_dict_bridge():
    from euromillioner_amd.models.mlp import DrawMLP

    net = DrawMLP((62, 32, 62), seed=3)
    layers = MS.layers_from_state_dict(net.state_dict())
    assert layers[0][0].shape == (62, 32)
    sd = MS.state_dict_from_layers(layers)
    for k, v in net.state_dict().items():
        assert torch.equal(sd[k], v)


def test_truncated_buffer_rejected():
    b = MS.nd4j_write(np.ones(10, np.float32))
    try:
        MS.nd4j_read(b[:-4])
    except ValueError:
        return
    raise AssertionError("truncated buffer accepted")
