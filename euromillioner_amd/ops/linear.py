"""Dense layers on the hand-written MFMA GEMM (``csrc/gemm.hip``, K1-K3) + fused loss (K10).

The reference's DL4J ``DenseLayer``/``OutputLayer`` stack (declared in ``pom.xml:62-66``,
never built) maps onto three GEMM shapes per layer, all served by one kernel template:

=========  ==========================================  ====================  ===========
pass       math                                         A / B layout          epilogue
=========  ==========================================  ====================  ===========
forward    ``Y = act(X W^T + b)``                       X [M,K] / W [N,K]     bias + act
dgrad      ``dZ_prev = (dZ W) * act'(Y_prev)``          dZ [M,N] / W [N,K]    act backward
wgrad      ``dW = dZ^T X``  (fp32, optional += )        dZ^T / X              alpha, beta
=========  ==========================================  ====================  ===========

Tensors handed to the kernel must have unit column stride, a row stride that is a
multiple of 8 elements and 16-byte aligned storage (one 16-byte vector per lane);
:func:`aligned` pads a copy when that does not hold (e.g. the 62-wide draw vectors).
"""
from __future__ import annotations

import torch

from . import _native as N

ACTS = {"none": 0, "identity": 0, "relu": 1, "sigmoid": 2, "tanh": 3}

N.register_signatures({
    "em_gemm_bf16": (N._i32, [N._c_void_p, N._i64, N._i32, N._c_void_p, N._i64, N._i32, N._c_void_p, N._i64, N._i32,
                              N._i32, N._i32, N._i32, N._c_void_p, N._i32, N._c_void_p, N._i64, N._i32, N._f32, N._f32,
                              N._c_void_p, N._i64, N._c_void_p]),
    "em_gemm_bf16_splitk": (N._i32, [N._c_void_p, N._i64, N._i32, N._c_void_p, N._i64, N._i32, N._c_void_p, N._i64,
                                     N._i32, N._i32, N._i32, N._i32, N._f32, N._i32, N._i32, N._i64, N._c_void_p]),
    "em_wgrad_skinny": (N._i32, [N._c_void_p, N._i64, N._c_void_p, N._i64, N._i32, N._i32, N._i32, N._c_void_p,
                                 N._i64, N._i32, N._f32, N._f32, N._c_void_p, N._i32, N._i32, N._c_void_p]),
    "em_gemm_bf16_cs": (N._i32, [N._c_void_p, N._i64, N._i32, N._c_void_p, N._i64, N._i32, N._c_void_p, N._i64,
                                 N._i32, N._i32, N._i32, N._i32, N._c_void_p, N._i32, N._c_void_p, N._i64, N._i32,
                                 N._f32, N._f32, N._c_void_p, N._i64, N._c_void_p, N._c_void_p]),
    "em_gemm_bf16_ex": (N._i32, [N._c_void_p, N._i64, N._i32, N._c_void_p, N._i64, N._i32, N._c_void_p, N._i64,
                                 N._i32, N._i32, N._i32, N._i32, N._c_void_p, N._i32, N._c_void_p, N._i64, N._i32,
                                 N._f32, N._f32, N._c_void_p, N._i64, N._c_void_p, N._c_void_p, N._c_void_p]),
    "em_colpart_reduce": (N._i32, [N._c_void_p, N._i32, N._i32, N._c_void_p, N._i32, N._f32, N._c_void_p]),
    "em_colsum_ws_floats": (N._i32, [N._i32, N._i32]),
    "em_colsum_bf16": (N._i32, [N._c_void_p, N._i64, N._i32, N._i32, N._c_void_p, N._i32, N._f32, N._c_void_p,
                                N._c_void_p]),
    "em_rowsum_bf16": (N._i32, [N._c_void_p, N._i64, N._i32, N._i32, N._c_void_p, N._i32, N._f32, N._c_void_p]),
    "em_transpose_bf16": (N._i32, [N._c_void_p, N._i64, N._i32, N._i32, N._c_void_p, N._i64, N._c_void_p]),
    "em_loss_grad": (N._i32, [N._c_void_p, N._i32, N._c_void_p, N._c_void_p, N._i64, N._i64, N._i32, N._f32,
                              N._c_void_p, N._i32, N._c_void_p, N._c_void_p, N._c_void_p]),
    "em_loss_grad_blocks": (N._i32, [N._i64]),
})


def round8(n: int) -> int:
    return (n + 7) // 8 * 8


def is_aligned(t: torch.Tensor) -> bool:
    return t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0


def aligned(t: torch.Tensor, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """Return ``t`` (cast to dtype) as a view with a GEMM-friendly layout, copying only if needed."""
    if t.dtype == dtype and is_aligned(t):
        return t
    r, c = t.shape
    buf = torch.zeros(r, round8(c), dtype=dtype, device=t.device)
    buf[:, :c] = t
    return buf[:, :c]


def empty_aligned(r: int, c: int, dtype: torch.dtype, device) -> torch.Tensor:
    return torch.empty(r, round8(c), dtype=dtype, device=device)[:, :c]


BIG_M, BIG_N, BIG_K = 256, 256, 64


def relu_bits(M: int, N_: int, device) -> torch.Tensor:
    """Buffer for the ReLU activity bits of an [M, N] activation (``gemm(bits=...)``): int32 [M / 32, N],
    bit m % 32 of word [m // 32, n] is ``act[m, n] > 0``."""
    if M % 32:
        raise ValueError("relu bits need M % 32 == 0")
    return torch.empty(M // 32, N_, dtype=torch.int32, device=device)


def big_ok(M: int, N_: int, K: int) -> bool:
    """Shapes the 256x256 kernel takes (otherwise the 128x128 any-layout kernel runs)."""
    return M % BIG_M == 0 and N_ % BIG_N == 0 and K % BIG_K == 0 and K > 0


def big_mn_ok(t: torch.Tensor, K: int) -> bool:
    """An MN-contiguous operand ([K, rows] storage) on the 256-tile path: 32-bit buffer offsets over K rows
    (``g_layout_ok`` in csrc/gemm.hip)."""
    return K * t.stride(0) * 2 < (1 << 31)


def gemm(a: torch.Tensor, a_kc: bool, b: torch.Tensor, b_kc: bool, out: torch.Tensor, M: int, N_: int, K: int,
         bias: torch.Tensor | None = None, act: str = "none", dact_src: torch.Tensor | None = None,
         dact: str = "relu", alpha: float = 1.0, beta: float = 0.0, ct: torch.Tensor | None = None,
         colpart: torch.Tensor | None = None, bits: torch.Tensor | None = None) -> torch.Tensor:
    """Raw K1-K3 launch.  ``a``/``b`` are bf16 in their storage shape; ``out`` fp32 or bf16 [M, N].
    ``ct`` (bf16 [N, M], 256-path only) receives a transposed copy of the output.
    ``colpart`` (fp32, >= M / 128 * N, 256-path only) receives the epilogue's column sums per 128 output
    rows (the fused bias gradient of a dgrad: ``colpart_reduce`` sums them).
    ``bits`` (:func:`relu_bits`, 256 path only): written by a bf16 forward with ``act="relu"``; read as
    act' by a ``dact="relu"`` dgrad given no ``dact_src`` (1 bit per element instead of the bf16 activation)."""
    for t, nm in ((a, "a"), (b, "b")):
        N.check_cuda(t, nm, torch.bfloat16, contiguous=False)
        if not is_aligned(t):
            raise ValueError(f"{nm}: needs unit column stride, row stride %8 and 16-byte alignment")
    N.check_cuda(out, "out", contiguous=False)
    if out.dtype not in (torch.float32, torch.bfloat16) or out.stride(1) != 1 or tuple(out.shape) != (M, N_):
        raise ValueError("out must be fp32/bf16 [M, N] with unit column stride")
    exp_a = (M, K) if a_kc else (K, M)
    exp_b = (N_, K) if b_kc else (K, N_)
    if tuple(a.shape) != exp_a or tuple(b.shape) != exp_b:
        raise ValueError(f"shape mismatch: a {tuple(a.shape)} vs {exp_a}, b {tuple(b.shape)} vs {exp_b}")
    if bias is not None:
        N.check_cuda(bias, "bias", torch.float32)
        if bias.numel() < N_:
            raise ValueError("bias too short")
    ldm = 0
    if dact_src is not None:
        N.check_cuda(dact_src, "dact_src", torch.bfloat16, contiguous=False)
        if tuple(dact_src.shape) != (M, N_) or dact_src.stride(1) != 1:
            raise ValueError("dact_src must be bf16 [M, N] with unit column stride")
        ldm = dact_src.stride(0)
    read_bits = bits is not None and dact_src is None and dact == "relu" and act in ("none", "identity")
    if bits is not None:
        N.check_cuda(bits, "bits", torch.int32)
        if not (read_bits or (act == "relu" and dact_src is None)):
            raise ValueError("bits: written by act='relu' or read by dact='relu' without dact_src")
        if (out.dtype != torch.bfloat16 or not (a_kc and big_ok(M, N_, K) and (b_kc or big_mn_ok(b, K)))
                or tuple(bits.shape) != (M // 32, N_)):
            raise ValueError("bits need the 256-tile path (A K-contiguous), a bf16 output and an int32 [M / 32, N] "
                             "buffer")
    if ct is not None:
        N.check_cuda(ct, "ct", torch.bfloat16, contiguous=False)
        if not (a_kc and b_kc and big_ok(M, N_, K)) or tuple(ct.shape) != (N_, M) or not is_aligned(ct):
            raise ValueError("ct needs the 256-tile NT path and an aligned bf16 [N, M] buffer")
    args = (a.data_ptr(), a.stride(0), int(a_kc), b.data_ptr(), b.stride(0), int(b_kc),
            out.data_ptr(), out.stride(0), int(out.dtype == torch.bfloat16), M, N_, K,
            bias.data_ptr() if bias is not None else None, ACTS[act],
            dact_src.data_ptr() if dact_src is not None else None, ldm,
            ACTS[dact] if (dact_src is not None or read_bits) else 0,
            float(alpha), float(beta), ct.data_ptr() if ct is not None else None, ct.stride(0) if ct is not None else 0)
    if colpart is not None:
        N.check_cuda(colpart, "colpart", torch.float32)
        if not (a_kc and big_ok(M, N_, K) and (b_kc or big_mn_ok(b, K))) or colpart.numel() < (M // 128) * N_:
            raise ValueError("colpart needs the 256-tile path (A K-contiguous) and M / 128 * N floats")
    if bits is not None:
        N.call("em_gemm_bf16_ex", *args, colpart.data_ptr() if colpart is not None else None, bits.data_ptr(),
               N.stream_handle(out.device))
    elif colpart is not None:
        N.call("em_gemm_bf16_cs", *args, colpart.data_ptr(), N.stream_handle(out.device))
    else:
        N.call("em_gemm_bf16", *args, N.stream_handle(out.device))
    return out


def colpart_reduce(part: torch.Tensor, nparts: int, n: int, out: torch.Tensor, accumulate: bool = False,
                   scale: float = 1.0) -> torch.Tensor:
    """``out[:n] (+)= scale * part.view(nparts, n).sum(0)`` in a fixed order (bias gradient from the
    partials a ``colpart`` GEMM wrote)."""
    N.check_cuda(part, "part", torch.float32)
    N.check_cuda(out, "out", torch.float32)
    if part.numel() < nparts * n or out.numel() < n:
        raise ValueError("colpart_reduce: buffer too small")
    N.call("em_colpart_reduce", part.data_ptr(), int(nparts), int(n), out.data_ptr(), int(accumulate), float(scale),
           N.stream_handle(out.device))
    return out


def transpose(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """bf16 [R, C] -> [C, R] (LDS-tiled, 16-B accesses)."""
    N.check_cuda(x, "x", torch.bfloat16, contiguous=False)
    if not is_aligned(x):
        x = aligned(x)
    R, Cc = x.shape
    if out is None:
        out = empty_aligned(Cc, R, torch.bfloat16, x.device)
    N.call("em_transpose_bf16", x.data_ptr(), x.stride(0), R, Cc, out.data_ptr(), out.stride(0),
           N.stream_handle(x.device))
    return out


def linear_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None, act: str = "none",
               out_dtype: torch.dtype = torch.bfloat16, out: torch.Tensor | None = None,
               ct: torch.Tensor | None = None, bits: torch.Tensor | None = None) -> torch.Tensor:
    """``act(x @ w.T + bias)``; x bf16 [M, K], w bf16 [N, K] (nn.Linear layout); ``ct`` gets the output^T,
    ``bits`` (relu) its activity bits."""
    M, K = x.shape
    N_ = w.shape[0]
    if out is None:
        out = empty_aligned(M, N_, out_dtype, x.device)
    return gemm(x, True, w, True, out, M, N_, K, bias=bias, act=act, ct=ct, bits=bits)


def linear_dgrad_nt(dz: torch.Tensor, wt: torch.Tensor, y_prev: torch.Tensor | None = None, dact: str = "relu",
                    out: torch.Tensor | None = None, ct: torch.Tensor | None = None,
                    colpart: torch.Tensor | None = None, bits: torch.Tensor | None = None) -> torch.Tensor:
    """dgrad from a transposed weight copy ``wt`` [K, N] (256-tile NT path): ``(dz @ wt.T) * act'(y_prev)``;
    ``colpart`` gets the bias-gradient partials of the result (see :func:`gemm`).  With ``bits`` (relu, from
    the forward that wrote y_prev) act' comes from the activity bits and y_prev is not read."""
    M, N_ = dz.shape
    K = wt.shape[0]
    if out is None:
        out = empty_aligned(M, K, torch.bfloat16, dz.device)
    if dact in ("none", "identity"):
        y_prev = bits = None
    if bits is not None:
        y_prev = None
    return gemm(dz, True, wt, True, out, M, K, N_, dact_src=y_prev, dact=dact, ct=ct, colpart=colpart, bits=bits)


def linear_wgrad_nt(dzt: torch.Tensor, xt: torch.Tensor, out: torch.Tensor | None = None,
                    beta: float = 0.0) -> torch.Tensor:
    """wgrad from transposed copies: ``dzt`` [N, M], ``xt`` [K, M] -> fp32 ``dzt @ xt.T (+ beta * out)`` [N, K]."""
    N_, M = dzt.shape
    K = xt.shape[0]
    if out is None:
        if beta != 0.0:
            raise ValueError("beta needs an existing out")
        out = empty_aligned(N_, K, torch.float32, dzt.device)
    return gemm(dzt, True, xt, True, out, N_, K, M, beta=beta)


def linear_dgrad(dz: torch.Tensor, w: torch.Tensor, y_prev: torch.Tensor | None = None, dact: str = "relu",
                 out: torch.Tensor | None = None, colpart: torch.Tensor | None = None,
                 bits: torch.Tensor | None = None) -> torch.Tensor:
    """``(dz @ w) * act'(y_prev)``; dz bf16 [M, N], w bf16 [N, K] -> bf16 [M, K]; ``colpart`` / ``bits`` as
    in :func:`linear_dgrad_nt` (256-tile shapes)."""
    M, N_ = dz.shape
    K = w.shape[1]
    if out is None:
        out = empty_aligned(M, K, torch.bfloat16, dz.device)
    if dact in ("none", "identity"):
        y_prev = bits = None
    if bits is not None:
        y_prev = None
    if big_ok(M, K, N_) and is_aligned(dz):
        # 256-tile shapes: transpose the (weight-sized) w once and take the NT path.  Reading w in place
        # (the kernel's MN-operand form, gemm(..., b_kc=False)) measured slower: 7.49 vs 6.72 ms at
        # 65536 x 8192 x 8192 -- its ds_read_b64_tr_b16 fragment reads double the LDS read instructions in
        # the ping-pong load segment (profiles/r5/gemm_mn_operands.txt); the transpose costs ~0.03 ms
        return gemm(dz, True, transpose(w), True, out, M, K, N_, dact_src=y_prev, dact=dact, colpart=colpart,
                    bits=bits)
    return gemm(dz, True, w, False, out, M, K, N_, dact_src=y_prev, dact=dact, colpart=colpart, bits=bits)


def linear_wgrad(dz: torch.Tensor, x: torch.Tensor, out: torch.Tensor | None = None, alpha: float = 1.0,
                 beta: float = 0.0, split_k: int | None = None) -> torch.Tensor:
    """``alpha * dz^T @ x (+ beta * out)`` in fp32; dz [M, N], x [M, K] bf16 -> [N, K].

    Small outputs with a huge reduction (e.g. 64 x 8192 over a 64k batch) are split over K
    (the batch) into fp32 partial slabs that are summed in a fixed order (deterministic)."""
    M, N_ = dz.shape
    K = x.shape[1]
    if out is None:
        out = empty_aligned(N_, K, torch.float32, dz.device)
    if split_k is None and _skinny_ok(dz, x, out):
        return _wgrad_skinny(dz, x, out, alpha, beta)
    if split_k is None and alpha == 1.0 and big_ok(N_, K, M) and out.dtype == torch.float32:
        # 256-tile shapes: both operands transposed to K-major (two LDS-tiled copies, ~0.45 ms each at
        # 65536 x 8192) and the NT path: 6.27 + 0.9 ms against 8.18 ms for the MN-operand form reading dz
        # and x in place (profiles/r5/gemm_mn_operands.txt)
        return gemm(transpose(dz), True, transpose(x), True, out, N_, K, M, beta=beta)
    tiles = ((N_ + 127) // 128) * ((K + 127) // 128)
    if split_k is None:
        split_k = 1
        if tiles < 256 and M >= 8192:
            split_k = max(1, min((1024 + tiles - 1) // tiles, M // 1024))
    if split_k <= 1:
        return gemm(dz, False, x, False, out, N_, K, M, alpha=alpha, beta=beta)
    for t, nm in ((dz, "dz"), (x, "x")):
        N.check_cuda(t, nm, torch.bfloat16, contiguous=False)
        if not is_aligned(t):
            raise ValueError(f"{nm}: needs an aligned bf16 layout")
    kstep = ((M + split_k - 1) // split_k + 63) // 64 * 64
    split_k = (M + kstep - 1) // kstep
    Kp = round8(K)
    parts = torch.empty(split_k, N_, Kp, dtype=torch.float32, device=dz.device)
    # one launch: blockIdx.y = K-slice -> its own fp32 partial [N, K]; then a fixed-order sum
    N.call("em_gemm_bf16_splitk", dz.data_ptr(), dz.stride(0), 0, x.data_ptr(), x.stride(0), 0, parts.data_ptr(), Kp,
           0, N_, K, M, float(alpha), split_k, kstep, N_ * Kp, N.stream_handle(dz.device))
    red = parts[:, :, :K].sum(0)
    if beta != 0.0:
        out.mul_(beta).add_(red)
    else:
        out.copy_(red)
    return out


def _skinny_ok(dz: torch.Tensor, x: torch.Tensor, out: torch.Tensor) -> bool:
    """64-wide x (batch >> 64) x 256k-wide weight gradients: the streaming skinny kernel."""
    M, N_ = dz.shape
    K = x.shape[1]
    narrow, wide = (N_, K) if N_ <= 64 else (K, N_)
    return (narrow <= 64 and wide % 256 == 0 and M % 64 == 0 and M >= 4096 and out.dtype == torch.float32
            and out.stride(1) == 1 and out.stride(0) % 8 == 0 and is_aligned(dz) and is_aligned(x))


def _wgrad_skinny(dz: torch.Tensor, x: torch.Tensor, out: torch.Tensor, alpha: float, beta: float) -> torch.Tensor:
    """``out = alpha * dz^T x (+ beta out)`` via em_wgrad_skinny: P = the 64-wide operand, Q = the wide
    one; the output is written transposed when dz is the wide side (first layer: [8192, 64])."""
    M, N_ = dz.shape
    trans = N_ > 64
    P, Q = (x, dz) if trans else (dz, x)
    J, W = P.shape[1], Q.shape[1]
    splits = max(1, min(256 // (W // 256), M // 64))
    kstep = ((M + splits - 1) // splits + 63) // 64 * 64
    while kstep * Q.stride(0) * 2 >= 1 << 31:  # 32-bit buffer offsets inside a K-slice
        splits *= 2
        kstep = ((M + splits - 1) // splits + 63) // 64 * 64
    splits = (M + kstep - 1) // kstep
    part = torch.empty(splits * 64 * W, dtype=torch.float32, device=dz.device)
    N.call("em_wgrad_skinny", P.data_ptr(), P.stride(0), Q.data_ptr(), Q.stride(0), M, J, W, out.data_ptr(),
           out.stride(0), int(trans), float(alpha), float(beta), part.data_ptr(), splits, kstep,
           N.stream_handle(dz.device))
    return out


def colsum(x: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False,
           scale: float = 1.0, ws: torch.Tensor | None = None) -> torch.Tensor:
    """Bias gradient: fp32 column sums of a bf16 [M, N] matrix (deterministic two-pass)."""
    N.check_cuda(x, "x", torch.bfloat16, contiguous=False)
    if not is_aligned(x):
        x = aligned(x)
    M, N_ = x.shape
    if out is None:
        out = torch.empty(N_, dtype=torch.float32, device=x.device)
    need = max(1, (M + 511) // 512 * N_)
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.float32, device=x.device)
    N.call("em_colsum_bf16", x.data_ptr(), x.stride(0), M, N_, out.data_ptr(), int(accumulate), float(scale),
           ws.data_ptr(), N.stream_handle(x.device))
    return out


def rowsum(x: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False,
           scale: float = 1.0) -> torch.Tensor:
    """fp32 row sums of a bf16 [R, C] matrix (bias gradient from a transposed dZ)."""
    N.check_cuda(x, "x", torch.bfloat16, contiguous=False)
    if not is_aligned(x):
        x = aligned(x)
    R, Cc = x.shape
    if out is None:
        out = torch.empty(R, dtype=torch.float32, device=x.device)
    N.call("em_rowsum_bf16", x.data_ptr(), x.stride(0), R, Cc, out.data_ptr(), int(accumulate), float(scale),
           N.stream_handle(x.device))
    return out


def loss_grad(logits: torch.Tensor, masks: torch.Tensor, B: int, loss: str = "softmax", offset: int = 0,
              sidx: torch.Tensor | None = None, grad_scale: float = 1.0, dz: torch.Tensor | None = None,
              partials: torch.Tensor | None = None,
              colpart: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """K10: (dz bf16 [B, 64] = grad_scale * dL/dlogits, per-block loss sums [ceil(B/4)]).
    ``colpart`` (fp32, >= loss_grad_blocks(B) * 64): per-block column sums of dz for the last layer's
    bias gradient (``colpart_reduce(colpart, loss_grad_blocks(B), 64, ...)``)."""
    from .fused_mlp import LOSS_KINDS, _check_draws

    _check_draws(masks, sidx, B, offset)
    N.check_cuda(logits, "logits", torch.float32, contiguous=False)
    if logits.stride(1) != 1 or logits.shape[1] < 62:
        raise ValueError("logits must be fp32 [B, >=62] with unit column stride")
    if dz is None:
        dz = torch.empty(B, 64, dtype=torch.bfloat16, device=logits.device)
    if partials is None:
        partials = torch.empty(max((B + 3) // 4, 1), dtype=torch.float32, device=logits.device)
    if colpart is not None:
        N.check_cuda(colpart, "colpart", torch.float32)
        if colpart.numel() < loss_grad_blocks(B) * 64:
            raise ValueError("colpart too small")
    N.call("em_loss_grad", logits.data_ptr(), logits.stride(0), masks.data_ptr(),
           sidx.data_ptr() if sidx is not None else None, B, offset, LOSS_KINDS[loss], float(grad_scale),
           dz.data_ptr(), dz.stride(0), partials.data_ptr(), colpart.data_ptr() if colpart is not None else None,
           N.stream_handle(logits.device))
    return dz, partials


def loss_grad_blocks(B: int) -> int:
    """Blocks (= colpart rows) of the K10 loss kernel for a batch of B."""
    return int(N.query("em_loss_grad_blocks", int(B)))


class _MLPFunction(torch.autograd.Function):
    """Whole-stack autograd node: saves each layer's bf16 input, fuses act' into dgrad."""

    @staticmethod
    def forward(ctx, x, act, *wb):
        ws, bs = wb[0::2], wb[1::2]
        wq = [aligned(w.detach()) for w in ws]
        h = aligned(x.detach())
        inputs = []
        for i, (w, b) in enumerate(zip(wq, bs)):
            last = i == len(wq) - 1
            inputs.append(h)
            h = linear_fwd(h, w, b.detach().float().contiguous(), "none" if last else act,
                           torch.float32 if last else torch.bfloat16)
        ctx.act = act
        ctx.wq = wq
        ctx.inputs = inputs
        ctx.shapes = [tuple(w.shape) for w in ws]
        return h

    @staticmethod
    def backward(ctx, gy):
        dz = aligned(gy)
        n = len(ctx.wq)
        grads = [None] * (2 * n)
        gx = None
        for i in reversed(range(n)):
            x_i = ctx.inputs[i]
            grads[2 * i] = linear_wgrad(dz, x_i)
            grads[2 * i + 1] = colsum(dz)
            if i > 0:
                dz = linear_dgrad(dz, ctx.wq[i], x_i, ctx.act)
            elif ctx.needs_input_grad[0]:
                gx = linear_dgrad(dz, ctx.wq[0]).float()
        ctx.inputs = None
        return (gx, None, *grads)


def mlp(x: torch.Tensor, weights, biases, activation: str = "relu") -> torch.Tensor:
    """Dense stack on the HIP kernels: hidden layers bf16 + act, last layer fp32 logits."""
    wb = []
    for w, b in zip(weights, biases):
        wb += [w, b]
    return _MLPFunction.apply(x, activation, *wb)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None, activation: str = "none",
           compute_dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """Single layer (no autograd through the kernel; use :func:`mlp` for training)."""
    del compute_dtype
    b = bias.detach().float().contiguous() if bias is not None else None
    return linear_fwd(aligned(x.detach()), aligned(weight.detach()), b, activation, torch.float32)
