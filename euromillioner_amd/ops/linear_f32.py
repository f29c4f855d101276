"""fp32 dense layers on the exact-fp32 MFMA GEMM (``csrc/gemm_f32.hip``) for ``--dtype fp32``.

Same three products per layer as :mod:`.linear` (forward with bias + activation, dgrad with the
activation backward fused, wgrad), fp32 end to end: the DL4J default data type of the reference's
declared network stack (``pom.xml:62-66``).  The small wgrad over a huge batch is split along K
(gridDim.y slices) and the slices summed, so it still fills 256 CUs.
"""
from __future__ import annotations

import torch

from . import _native as N
from .linear import ACTS

N.register_signatures({
    "em_gemm_f32": (N._i32, [N._c_void_p, N._i64, N._i32, N._c_void_p, N._i64, N._i32, N._c_void_p, N._i64,
                             N._i32, N._i32, N._i32, N._c_void_p, N._i32, N._c_void_p, N._i64, N._i32, N._f32, N._f32,
                             N._i32, N._i32, N._i64, N._c_void_p, N._c_void_p]),
    "em_onehot_encode_f32": (N._i32, [N._c_void_p, N._c_void_p, N._i64, N._i64, N._i32, N._i32, N._c_void_p,
                                      N._c_void_p]),
    "em_loss_grad_f32": (N._i32, [N._c_void_p, N._i32, N._c_void_p, N._c_void_p, N._i64, N._i64, N._i32, N._f32,
                                  N._c_void_p, N._i32, N._c_void_p, N._c_void_p, N._c_void_p]),
})

TILE = 128


def _check2d(t: torch.Tensor, name: str):
    N.check_cuda(t, name, torch.float32, contiguous=False)
    if t.dim() != 2 or (t.stride(1) != 1 and t.shape[1] != 1):
        raise ValueError(f"{name}: needs a 2-D fp32 tensor with unit column stride")


def gemm_f32(a: torch.Tensor, a_kc: bool, b: torch.Tensor, b_kc: bool, out: torch.Tensor, M: int, N_: int, K: int,
             bias: torch.Tensor | None = None, act: str = "none", dact_src: torch.Tensor | None = None,
             dact: str = "relu", alpha: float = 1.0, beta: float = 0.0, splits: int = 1,
             parts: torch.Tensor | None = None, colpart: torch.Tensor | None = None) -> torch.Tensor:
    """Raw launch.  ``splits > 1`` (no bias/act/dact): K is cut into slices written to ``parts``
    ([splits, M, N] fp32) and summed into ``out`` (``out = alpha * sum + beta * out``).
    ``colpart`` (splits == 1, fp32 >= ceil(M / 128) * N): per-128-row column sums of ``out``."""
    _check2d(a, "a")
    _check2d(b, "b")
    _check2d(out, "out")
    if tuple(a.shape) != ((M, K) if a_kc else (K, M)) or tuple(b.shape) != ((N_, K) if b_kc else (K, N_)):
        raise ValueError(f"shape mismatch: a {tuple(a.shape)}, b {tuple(b.shape)} for M={M} N={N_} K={K}")
    if tuple(out.shape) != (M, N_):
        raise ValueError("out must be [M, N]")
    if bias is not None:
        N.check_cuda(bias, "bias", torch.float32)
        if bias.numel() < N_:
            raise ValueError("bias too short")
    ldy = 0
    if dact_src is not None:
        _check2d(dact_src, "dact_src")
        if tuple(dact_src.shape) != (M, N_):
            raise ValueError("dact_src must be [M, N]")
        ldy = dact_src.stride(0)
    st = N.stream_handle(out.device)
    if colpart is not None:
        N.check_cuda(colpart, "colpart", torch.float32)
        if splits > 1 or colpart.numel() < -(-M // TILE) * N_:
            raise ValueError("colpart needs splits == 1 and ceil(M / 128) * N floats")
    if splits > 1:
        if bias is not None or act != "none" or dact_src is not None:
            raise ValueError("split-K takes no epilogue")
        kstep = -(-K // splits)
        if parts is None or tuple(parts.shape) != (splits, M, N_) or not parts.is_contiguous():
            parts = torch.empty(splits, M, N_, dtype=torch.float32, device=out.device)
        N.call("em_gemm_f32", a.data_ptr(), a.stride(0), int(a_kc), b.data_ptr(), b.stride(0), int(b_kc),
               parts.data_ptr(), N_, M, N_, K, None, 0, None, 0, 0, float(alpha), 0.0, splits, kstep, M * N_, None,
               st)
        if beta == 0.0:
            torch.sum(parts, dim=0, out=out) if out.is_contiguous() else out.copy_(parts.sum(0))
        else:
            out.mul_(beta).add_(parts.sum(0))
        return out
    N.call("em_gemm_f32", a.data_ptr(), a.stride(0), int(a_kc), b.data_ptr(), b.stride(0), int(b_kc),
           out.data_ptr(), out.stride(0), M, N_, K, bias.data_ptr() if bias is not None else None,
           ACTS[dact] if dact_src is not None else ACTS[act],  # with dact_src the kernel's act names act'
           dact_src.data_ptr() if dact_src is not None else None, ldy, int(dact_src is not None),
           float(alpha), float(beta), 1, 0, 0, colpart.data_ptr() if colpart is not None else None, st)
    return out


def linear_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None, act: str, out: torch.Tensor) -> torch.Tensor:
    """``out = act(x @ w.T + bias)``; x [M, K], w [N, K]."""
    M, K = x.shape
    return gemm_f32(x, True, w, True, out, M, w.shape[0], K, bias=bias, act=act)


def linear_dgrad(dz: torch.Tensor, w: torch.Tensor, y_prev: torch.Tensor, act: str, out: torch.Tensor,
                 colpart: torch.Tensor | None = None) -> torch.Tensor:
    """``out = (dz @ w) * act'(y_prev)``; dz [M, N], w [N, K] (k-major as the B operand).  ``colpart``:
    per-128-row column sums of ``out`` (the previous layer's bias gradient, ``colpart_reduce``)."""
    M, Nn = dz.shape
    return gemm_f32(dz, True, w, False, out, M, w.shape[1], Nn, dact_src=y_prev, dact=act, colpart=colpart)


def linear_wgrad(dz: torch.Tensor, x: torch.Tensor, out: torch.Tensor, parts_cache: dict | None = None) -> torch.Tensor:
    """``out = dz.T @ x`` (fp32 [N, K]); the batch is the reduction axis -> split-K for small layers."""
    B, Nn = dz.shape
    K = x.shape[1]
    tiles = -(-Nn // TILE) * -(-K // TILE)
    splits = 1
    if tiles < 256 and B >= 4096:
        splits = max(1, min(-(-1024 // tiles), B // 2048))
    parts = None
    if splits > 1 and parts_cache is not None:
        key = (splits, Nn, K)
        parts = parts_cache.get(key)
        if parts is None:
            parts = parts_cache[key] = torch.empty(splits, Nn, K, dtype=torch.float32, device=dz.device)
    return gemm_f32(dz, False, x, False, out, Nn, K, B, splits=splits, parts=parts)


def onehot(draws: torch.Tensor, B: int, offset: int = 0, which: int = 0, sidx: torch.Tensor | None = None,
           out: torch.Tensor | None = None) -> torch.Tensor:
    """K14, fp32 output: multi-hot [B, 64] of draws[idx + which]."""
    from . import fused_mlp as FM

    FM._check_draws(draws, sidx, B, offset, need_next=(which == 1))
    if out is None:
        out = torch.empty(B, 64, dtype=torch.float32, device=draws.device)
    N.call("em_onehot_encode_f32", draws.data_ptr(), sidx.data_ptr() if sidx is not None else None, B, offset, which,
           0, out.data_ptr(), N.stream_handle(draws.device))
    return out


def loss_grad(logits: torch.Tensor, masks: torch.Tensor, B: int, loss: str, offset: int = 0,
              sidx: torch.Tensor | None = None, grad_scale: float = 1.0, dz: torch.Tensor | None = None,
              partials: torch.Tensor | None = None, colpart: torch.Tensor | None = None):
    """K10 with an fp32 dL/dlogits [B, 64] (pre-scaled); returns (dz, per-block loss sums).
    ``colpart``: per-block column sums of dz (see ``linear.loss_grad``)."""
    from . import fused_mlp as FM

    _check2d(logits, "logits")
    if dz is None:
        dz = torch.empty(B, 64, dtype=torch.float32, device=logits.device)
    if partials is None:
        partials = torch.empty((B + 3) // 4, dtype=torch.float32, device=logits.device)
    N.call("em_loss_grad_f32", logits.data_ptr(), logits.stride(0), masks.data_ptr(),
           sidx.data_ptr() if sidx is not None else None, B, offset, FM.LOSS_KINDS[loss], float(grad_scale),
           dz.data_ptr(), dz.stride(0), partials.data_ptr(), colpart.data_ptr() if colpart is not None else None,
           N.stream_handle(logits.device))
    return dz, partials[:(B + 3) // 4]
