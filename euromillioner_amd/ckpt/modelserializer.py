"""DL4J ``ModelSerializer``-layout checkpoints for the MLPs (T6, north star N9).

The reference pins DL4J 0.9.1 (``pom.xml:62-66``) but never saves a model; the north
star asks for its checkpoint format.  A DL4J ``ModelSerializer.writeModel(net, file,
saveUpdater)`` zip holds:

``configuration.json``
    the ``MultiLayerConfiguration`` JSON (confs[] with one ``layer`` per DenseLayer /
    OutputLayer: nIn, nOut, activationFn, lossFn, updater; plus backprop settings).
``coefficients.bin``
    the flattened parameter row vector written by ``Nd4j.write``: the shape-info
    buffer, then the data buffer.  Each buffer is a Java ``DataOutputStream``
    (big-endian): ``writeUTF(allocationMode)``, ``writeInt(length)``,
    ``writeUTF(dataType)``, then the elements.  Per layer the order is **W** (nIn x
    nOut, Fortran order) then **b** (1 x nOut).
``updaterState.bin`` (optional)
    the Adam state view, same encoding: [m (all params) | v (all params)] for the one
    updater block.
``normalizer.bin`` is not written (no normaliser).  We also add ``euromillioner.json``
(step counter, loss choice, data provenance) which DL4J ignores.

This byte layout cannot be checked against a real DL4J artifact offline (no
network, no JVM here): it is pinned by ``tests/test_ckpt.py`` golden tests and the
assumptions are the ones listed above ("parity unpinned" w.r.t. real DL4J).
"""
from __future__ import annotations

import io
import json
import struct
import zipfile

import numpy as np

ALLOC_MODE = "HEAP"


def _write_utf(buf: io.BytesIO, s: str) -> None:
    b = s.encode("utf-8")  # modified UTF-8 == UTF-8 for ASCII
    buf.write(struct.pack(">H", len(b)))
    buf.write(b)


def _read_utf(buf: io.BytesIO) -> str:
    (n,) = struct.unpack(">H", buf.read(2))
    return buf.read(n).decode("utf-8")


def _write_buffer(buf: io.BytesIO, data: np.ndarray, dtype: str) -> None:
    _write_utf(buf, ALLOC_MODE)
    buf.write(struct.pack(">i", int(data.size)))
    _write_utf(buf, dtype)
    fmt = {"INT": ">i4", "FLOAT": ">f4", "DOUBLE": ">f8", "LONG": ">i8"}[dtype]
    buf.write(np.ascontiguousarray(data, dtype=fmt).tobytes())


def _read_buffer(buf: io.BytesIO) -> np.ndarray:
    _read_utf(buf)  # allocation mode
    (n,) = struct.unpack(">i", buf.read(4))
    dtype = _read_utf(buf)
    fmt = {"INT": ">i4", "FLOAT": ">f4", "DOUBLE": ">f8", "LONG": ">i8"}[dtype]
    raw = buf.read(n * np.dtype(fmt).itemsize)
    if len(raw) != n * np.dtype(fmt).itemsize:
        raise ValueError("truncated ND4J buffer")
    return np.frombuffer(raw, dtype=fmt)


def nd4j_write(vec: np.ndarray) -> bytes:
    """``Nd4j.write`` of a [1, N] row vector in 'c' order (float)."""
    v = np.asarray(vec, dtype=np.float32).reshape(-1)
    n = v.size
    shape_info = np.array([2, 1, n, n, 1, 0, 1, ord("c")], dtype=np.int32)  # rank, shape, stride, offset, ews, order
    b = io.BytesIO()
    _write_buffer(b, shape_info, "INT")
    _write_buffer(b, v, "FLOAT")
    return b.getvalue()


def nd4j_read(data: bytes) -> np.ndarray:
    b = io.BytesIO(data)
    shape_info = _read_buffer(b).astype(np.int64)
    vals = _read_buffer(b).astype(np.float32)
    rank = int(shape_info[0])
    shape = tuple(int(x) for x in shape_info[1:1 + rank])
    if int(np.prod(shape)) != vals.size:
        raise ValueError("corrupt ND4J buffer: shape/length mismatch")
    return vals.reshape(-1)


def flatten_params(layers: list[tuple[np.ndarray, np.ndarray]]) -> np.ndarray:
    """layers: [(W [nIn, nOut], b [nOut])] -> DL4J flat view (W in Fortran order, then b)."""
    out = []
    for W, b in layers:
        out.append(np.asarray(W, np.float32).reshape(-1, order="F"))
        out.append(np.asarray(b, np.float32).reshape(-1))
    return np.concatenate(out) if out else np.zeros(0, np.float32)


def unflatten_params(flat: np.ndarray, sizes: list[int]) -> list[tuple[np.ndarray, np.ndarray]]:
    out, off = [], 0
    for nin, nout in zip(sizes[:-1], sizes[1:]):
        W = flat[off:off + nin * nout].reshape((nin, nout), order="F")
        off += nin * nout
        b = flat[off:off + nout]
        off += nout
        out.append((W.copy(), b.copy()))
    if off != flat.size:
        raise ValueError(f"parameter count mismatch: {off} != {flat.size}")
    return out


def multilayer_configuration(sizes: list[int], activation: str = "relu", loss: str = "softmax", lr: float = 1e-3,
                             betas=(0.9, 0.999), eps: float = 1e-8, seed: int = 0) -> dict:
    """A DL4J 0.9.1-style MultiLayerConfiguration JSON for Dense(...)+Output layers."""
    act_name = {"relu": "ReLU", "sigmoid": "Sigmoid", "tanh": "TanH", "identity": "Identity"}[activation]
    loss_fn = {"softmax": ("LossMCXENT", "Softmax"), "bce": ("LossBinaryXENT", "Sigmoid")}[loss]
    updater = {"@class": "org.nd4j.linalg.learning.config.Adam", "learningRate": lr, "beta1": betas[0],
               "beta2": betas[1], "epsilon": eps}
    confs = []
    for i, (nin, nout) in enumerate(zip(sizes[:-1], sizes[1:])):
        last = i == len(sizes) - 2
        layer = {"@class": "org.deeplearning4j.nn.conf.layers." + ("OutputLayer" if last else "DenseLayer"),
                 "layerName": f"layer{i}", "nin": int(nin), "nout": int(nout),
                 "activationFn": {"@class": "org.nd4j.linalg.activations.impl.Activation" +
                                  (loss_fn[1] if last else act_name)},
                 "weightInit": "XAVIER", "biasInit": 0.0, "iupdater": updater}
        if last:
            layer["lossFn"] = {"@class": "org.nd4j.linalg.lossfunctions.impl." + loss_fn[0]}
            if loss == "softmax":
                layer["euromillionerGroups"] = [[0, 50], [50, 62]]  # grouped softmax (50 main / 12 stars)
        confs.append({"layer": layer, "seed": seed, "miniBatch": True, "optimizationAlgo":
                      "STOCHASTIC_GRADIENT_DESCENT", "pretrain": False, "iterationCount": 0})
    return {"backprop": True, "backpropType": "Standard", "confs": confs, "pretrain": False,
            "tbpttBackLength": 20, "tbpttFwdLength": 20, "inputPreProcessors": {}}


def save(path: str, layers: list[tuple[np.ndarray, np.ndarray]], config: dict, updater_m: np.ndarray | None = None,
         updater_v: np.ndarray | None = None, extra: dict | None = None) -> None:
    flat = flatten_params(layers)
    with zipfile.ZipFile(path, "w", compression=zipfile.ZIP_DEFLATED) as z:
        z.writestr("configuration.json", json.dumps(config, indent=2))
        z.writestr("coefficients.bin", nd4j_write(flat))
        if updater_m is not None and updater_v is not None:
            st = np.concatenate([np.asarray(updater_m, np.float32).reshape(-1),
                                 np.asarray(updater_v, np.float32).reshape(-1)])
            z.writestr("updaterState.bin", nd4j_write(st))
        if extra is not None:
            z.writestr("euromillioner.json", json.dumps(extra, indent=2, default=float))


def load(path: str) -> dict:
    with zipfile.ZipFile(path) as z:
        names = set(z.namelist())
        cfg = json.loads(z.read("configuration.json"))
        flat = nd4j_read(z.read("coefficients.bin"))
        sizes = [cfg["confs"][0]["layer"]["nin"]] + [c["layer"]["nout"] for c in cfg["confs"]]
        out = {"config": cfg, "sizes": sizes, "layers": unflatten_params(flat, sizes), "flat": flat}
        if "updaterState.bin" in names:
            st = nd4j_read(z.read("updaterState.bin"))
            half = st.size // 2
            out["m"], out["v"] = st[:half], st[half:]
        if "euromillioner.json" in names:
            out["extra"] = json.loads(z.read("euromillioner.json"))
    return out


# ---- bridges to our models -------------------------------------------------------------------
def layers_from_state_dict(sd: dict) -> list[tuple[np.ndarray, np.ndarray]]:
    """nn.Linear-style state dict (weight [out, in]) -> DL4J (W [in, out], b)."""
    idx = sorted({k.split(".")[0] + "." + k.split(".")[1] if k.startswith("layers.") else k.split(".")[0]
                  for k in sd if k.endswith(".weight")}, key=_layer_key)
    out = []
    for p in idx:
        out.append((sd[p + ".weight"].detach().cpu().numpy().T.astype(np.float32),
                    sd[p + ".bias"].detach().cpu().numpy().astype(np.float32)))
    return out


def _layer_key(name: str):
    tail = name.split(".")[-1]
    digits = "".join(ch for ch in tail if ch.isdigit())
    return int(digits) if digits else 0


def state_dict_from_layers(layers, prefix: str = "layers") -> dict:
    import torch

    sd = {}
    for i, (W, b) in enumerate(layers):
        sd[f"{prefix}.{i}.weight"] = torch.from_numpy(np.ascontiguousarray(W.T))
        sd[f"{prefix}.{i}.bias"] = torch.from_numpy(np.ascontiguousarray(b))
    return sd
