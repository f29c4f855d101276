"""Python face of the random-forest kernels (``csrc/forest.hip``: K8 hist, K9 split scan,
K10 partition, K11 predict) and their native level-wise driver ``em_rf_fit``.

The reference only declares Spark MLlib's RandomForest (``/root/reference/pom.xml:56-61``,
``README.md:6``); SURVEY.md §2.4 N7 / BASELINE config 4 define the 100-tree one-hot forest."""
from __future__ import annotations

import numpy as np
import torch

from . import _native as N

N.register_signatures({
    "em_rf_nodes": (N._i32, [N._i32]),
    "em_rf_row_bytes": (N._i32, [N._i32, N._i32, N._i64]),
    "em_rf_acc_words": (N._i64, [N._i32, N._i32, N._i32]),
    "em_rf_fit": (N._i32, [N._c_void_p, N._i32, N._c_void_p, N._i64, N._i32, N._i32, N._i32, N._i32, N._i32, N._i32,
                           N.ctypes.c_uint64, N._i32, N._c_void_p, N._c_void_p, N._c_void_p, N._c_void_p, N._c_void_p,
                           N._c_void_p, N._c_void_p, N._c_void_p, N._c_void_p, N._c_void_p, N._c_void_p,
                           N._c_void_p]),
    "em_rf_predict": (N._i32, [N._c_void_p, N._i32, N._i64, N._c_void_p, N._c_void_p, N._i32, N._i32, N._i32,
                               N._c_void_p, N._i32, N._c_void_p, N._c_void_p]),
    "em_rf_predict_scratch": (N._i64, [N._i32, N._i32, N._i32]),
})


def _u64_to_device(a: np.ndarray, device) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(device)


def fit(X: np.ndarray | torch.Tensor, Y: np.ndarray | torch.Tensor, F: int, t_off: int, T: int, max_depth: int,
        k: int, min_leaf: int, bootstrap: bool, seed: int, device="cuda", return_device: bool = False):
    """Grow trees [t_off, t_off+T) on the GPU; returns (feat, value, gain, cover) numpy arrays."""
    dev = torch.device(device)
    Xd = X if isinstance(X, torch.Tensor) else _u64_to_device(X, dev)
    Yd = Y if isinstance(Y, torch.Tensor) else _u64_to_device(Y, dev)
    n = Xd.shape[0]
    W = Xd.shape[1] if Xd.dim() == 2 else 1
    if Yd.numel() != n:
        raise ValueError("X and Y row counts differ")
    if n >= 2**31 - 1 or n < 1:
        raise ValueError("rows must be in [1, 2^31-2]")
    nodes = (1 << (max_depth + 1)) - 1
    # per-tree row lists: 16-B records (x, y, weight) for one-word features, else int32 row ids
    rw = N.query("em_rf_row_bytes", W, F, n) // 4
    rows_a = torch.empty(T, n, rw, dtype=torch.int32, device=dev)
    rows_b = torch.empty(T, n, rw, dtype=torch.int32, device=dev)
    seg = torch.empty(T, nodes, 2, dtype=torch.int32, device=dev)
    feat = torch.full((T, nodes), -2, dtype=torch.int16, device=dev)
    value = torch.zeros(T, nodes, 64, dtype=torch.float32, device=dev)
    gain = torch.zeros(T, nodes, dtype=torch.float64, device=dev)
    cover = torch.zeros(T, nodes, dtype=torch.float32, device=dev)
    # per-level scratch: candidate lists, per-node integer sums, partition counters
    acc_words = N.query("em_rf_acc_words", T, max_depth, k)
    if acc_words < 0:
        raise ValueError("unsupported forest shape (trees / depth / candidate count)")
    cand = torch.empty(T, 1 << max_depth, k, dtype=torch.int16, device=dev)
    acc = torch.empty(acc_words, dtype=torch.int32, device=dev)
    lrc = torch.empty(T, 1 << max_depth, 2, dtype=torch.int32, device=dev)
    wl = torch.empty(T * (1 << max_depth) + 1, dtype=torch.int32, device=dev)  # per-level work list
    N.call("em_rf_fit", Xd.data_ptr(), W, Yd.data_ptr(), n, F, T, max_depth, k, min_leaf, int(bootstrap),
           int(seed) & 0xFFFFFFFFFFFFFFFF, int(t_off), rows_a.data_ptr(), rows_b.data_ptr(), seg.data_ptr(),
           feat.data_ptr(), value.data_ptr(), gain.data_ptr(), cover.data_ptr(), cand.data_ptr(), acc.data_ptr(),
           lrc.data_ptr(), wl.data_ptr(), N.stream_handle(dev))
    del rows_a, rows_b, cand, acc, lrc, wl
    if return_device:
        return feat, value, gain, cover
    return feat.cpu().numpy(), value.cpu().numpy(), gain.cpu().numpy(), cover.cpu().numpy()


def predict(X, feat, value, max_depth: int, out_logit: bool = False, device="cuda", stream_trees: bool = True
            ) -> torch.Tensor:
    """K11: mean leaf vector per row -> [N, 64] fp32 (probabilities, or logits if out_logit).
    ``stream_trees``: single-word rows and depth <= 8 stream the trees through LDS (csrc/forest.hip
    rf_predict_lds, bit-identical); False forces the one-wave-per-row kernel."""
    dev = torch.device(device)
    Xd = X if isinstance(X, torch.Tensor) else _u64_to_device(X, dev)
    n = Xd.shape[0]
    W = Xd.shape[1] if Xd.dim() == 2 else 1
    fd = feat if isinstance(feat, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(feat)).to(dev)
    vd = value if isinstance(value, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(value)).to(dev)
    T = fd.shape[0]
    if fd.shape[1] != (1 << (max_depth + 1)) - 1:
        raise ValueError("feat does not match max_depth")
    out = torch.empty(n, 64, dtype=torch.float32, device=dev)
    nb = N.lib().em_rf_predict_scratch(W, T, max_depth) if stream_trees else 0
    prep = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev) if nb > 0 else None
    N.call("em_rf_predict", Xd.data_ptr(), W, n, fd.data_ptr(), vd.data_ptr(), T, max_depth, int(out_logit),
           out.data_ptr(), 64, prep.data_ptr() if prep is not None else None, N.stream_handle(dev))
    return out
