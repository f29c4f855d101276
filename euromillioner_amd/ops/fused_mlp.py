"""Python face of the fused small-MLP kernels (``csrc/mlp_fused.hip``, ``csrc/adam.hip``,
``csrc/metrics.hip``): the 62->128->62 MLP the reference declares through DL4J but never builds
(``/root/reference/pom.xml:62-66``, ``README.md:2,6``; BASELINE.json configs 1-3).

Flat fp32 parameter layout (``P = 16448`` floats; the pads stay exactly 0):

=========  ===============  =================================================
offset     shape            meaning
=========  ===============  =================================================
0          W1 [64][128]     rows 0..61 = Linear(62,128).weight^T, row 62 = b1
8192       W2 [128][64]     cols 0..61 = Linear(128,62).weight^T
16384      b2 [64]          0..61 = Linear(128,62).bias
=========  ===============  =================================================
"""
from __future__ import annotations

import torch

from . import _native as N

IN, HID, OUT = 64, 128, 64
P_W1, P_W2, P_B2 = 0, IN * HID, IN * HID + HID * OUT
P_TOTAL = P_B2 + OUT
IMG_BYTES = 54528  # == em_mlp_fused_image_bytes() (csrc/mlp_fused.hip, padded weight images)
SLAB_STRIDE = 16640  # floats between per-workgroup gradient slabs (csrc/mlp_fused.hip)
LOSS_KINDS = {"softmax": 0, "bce": 1}


def unflatten(flat: torch.Tensor) -> dict[str, torch.Tensor]:
    """Logical (PyTorch nn.Linear-shaped) views of the flat buffer."""
    W1 = flat[P_W1:P_W2].view(IN, HID)
    W2 = flat[P_W2:P_B2].view(HID, OUT)
    b2 = flat[P_B2:P_TOTAL]
    return {
        "l1.weight": W1[:62].t(),  # [128, 62]
        "l1.bias": W1[62],  # [128]
        "l2.weight": W2[:, :62].t(),  # [62, 128]
        "l2.bias": b2[:62],  # [62]
    }


def flatten(sd: dict[str, torch.Tensor], device=None) -> torch.Tensor:
    flat = torch.zeros(P_TOTAL, dtype=torch.float32, device=device)
    W1 = flat[P_W1:P_W2].view(IN, HID)
    W2 = flat[P_W2:P_B2].view(HID, OUT)
    W1[:62] = sd["l1.weight"].t().to(flat)
    W1[62] = sd["l1.bias"].to(flat)
    W2[:, :62] = sd["l2.weight"].t().to(flat)
    flat[P_B2:P_B2 + 62] = sd["l2.bias"].to(flat)
    return flat


def pad_mask(device=None) -> torch.Tensor:
    """1 for real parameters, 0 for the padding slots."""
    m = torch.zeros(P_TOTAL, dtype=torch.float32, device=device)
    m[P_W1:P_W2].view(IN, HID)[:63] = 1
    m[P_W2:P_B2].view(HID, OUT)[:, :62] = 1
    m[P_B2:P_B2 + 62] = 1
    return m


def pack(params: torch.Tensor, img: torch.Tensor) -> None:
    N.check_cuda(params, "params", torch.float32)
    N.check_cuda(img, "img", torch.uint8)
    if params.numel() != P_TOTAL or img.numel() < IMG_BYTES:
        raise ValueError("bad params/img size")
    N.call("em_mlp_fused_pack", params.data_ptr(), img.data_ptr(), N.stream_handle(params.device))


def rows_to_masks(rows: torch.Tensor) -> torch.Tensor:
    """[N, 8] uint8 draw rows (GPU) -> [N] int64 (bit pattern = uint64 feature mask).

    Every draw kernel reads samples in this format: bit n-1 = main number n,
    bit 49+s = star s (the bias feature 62 is added in-kernel)."""
    N.check_cuda(rows, "rows", torch.uint8)
    if rows.dim() != 2 or rows.shape[1] != 8:
        raise ValueError("rows must be [N, 8] uint8")
    out = torch.empty(rows.shape[0], dtype=torch.int64, device=rows.device)
    N.call("em_rows_to_masks", rows.data_ptr(), rows.shape[0], out.data_ptr(), N.stream_handle(rows.device))
    return out


def masks_from_numpy(numbers, device) -> torch.Tensor:
    """Host path: numpy [N, 8] rows -> device int64 masks (via data.draws.mask_bits)."""
    from ..data.draws import mask_bits

    return torch.from_numpy(mask_bits(numbers).view("int64")).to(device)


def _check_draws(draws: torch.Tensor, sidx: torch.Tensor | None, B: int, offset: int, need_next: bool = True):
    N.check_cuda(draws, "masks", torch.int64)
    if draws.dim() != 1:
        raise ValueError("masks must be a 1-D int64 tensor of feature masks (see rows_to_masks)")
    n = draws.shape[0]
    if B >= 2**31 - 1:
        raise ValueError("at most 2^31-2 samples per step")
    if sidx is not None:
        if n >= 2**31 - 1:
            raise ValueError("sample_idx addressing covers at most 2^31-2 draws (use sequential offsets)")
        N.check_cuda(sidx, "sample_idx", torch.int32)
        if sidx.numel() < B:
            raise ValueError("sample_idx shorter than B")
        if B > 0:
            lo, hi = int(sidx[:B].min()), int(sidx[:B].max())
            if lo < 0 or hi + (1 if need_next else 0) >= n:
                raise ValueError("sample_idx out of range")
    elif B > 0 and (offset < 0 or offset + B - 1 + (1 if need_next else 0) >= n):
        raise ValueError(f"samples [{offset}, {offset + B}) + next draw exceed {n} draws")


ADAM_PRE = 4  # em_adam_slab mode bit: step counter already advanced by the train kernel (csrc/adam.hip)


def train_partials(draws: torch.Tensor, B: int, img: torch.Tensor, slabs: torch.Tensor, loss_slabs: torch.Tensor,
                   loss: str = "softmax", offset: int = 0, sidx: torch.Tensor | None = None,
                   check: bool = True, step: torch.Tensor | None = None) -> int:
    """Launch K7: per-workgroup gradient slabs for B samples.  Returns the grid size used.
    ``step`` (the optimizer's int32 state) is advanced by one in the same launch; the Adam launch
    that consumes these slabs must then pass ``pre=True``."""
    if check:
        _check_draws(draws, sidx, B, offset)
        N.check_cuda(img, "img", torch.uint8)
        N.check_cuda(slabs, "slabs", torch.float32)
        N.check_cuda(loss_slabs, "loss_slabs", torch.float32)
        if slabs.dim() != 2 or slabs.shape[1] != SLAB_STRIDE or loss_slabs.numel() < slabs.shape[0]:
            raise ValueError("slabs must be [nslab, SLAB_STRIDE]")
    groups = (B + 127) // 128
    nslab = max(1, min(slabs.shape[0], groups))
    N.call("em_mlp_fused_train", draws.data_ptr(), sidx.data_ptr() if sidx is not None else None, B, offset,
           img.data_ptr(), slabs.data_ptr(), loss_slabs.data_ptr(), nslab, LOSS_KINDS[loss],
           step.data_ptr() if step is not None else None, N.stream_handle(draws.device))
    return nslab


def train_partials_f32(draws: torch.Tensor, B: int, params: torch.Tensor, slabs: torch.Tensor,
                       loss_slabs: torch.Tensor, loss: str = "softmax", offset: int = 0,
                       sidx: torch.Tensor | None = None, check: bool = True, step: torch.Tensor | None = None) -> int:
    """:func:`train_partials` in exact fp32 (``csrc/mlp_fused_f32.hip``: every product a
    v_mfma_f32_32x32x2_f32): reads the fp32 master ``params`` instead of the bf16 weight images and
    writes the same per-workgroup gradient slabs.  Returns the grid size used."""
    if check:
        _check_draws(draws, sidx, B, offset)
        N.check_cuda(params, "params", torch.float32)
        if params.numel() != P_TOTAL:
            raise ValueError("params must hold P_TOTAL floats")
        if slabs.dim() != 2 or slabs.shape[1] != SLAB_STRIDE or loss_slabs.numel() < slabs.shape[0]:
            raise ValueError("slabs must be [nslab, SLAB_STRIDE]")
    nslab = max(1, min(slabs.shape[0], (B + 127) // 128))
    N.call("em_mlp_fused_train_f32", draws.data_ptr(), sidx.data_ptr() if sidx is not None else None, B, offset,
           params.data_ptr(), slabs.data_ptr(), loss_slabs.data_ptr(), nslab, LOSS_KINDS[loss],
           step.data_ptr() if step is not None else None, N.stream_handle(draws.device))
    return nslab


def forward_logits(draws: torch.Tensor, B: int, img: torch.Tensor, out: torch.Tensor | None = None, offset: int = 0,
                   sidx: torch.Tensor | None = None) -> torch.Tensor:
    _check_draws(draws, sidx, B, offset, need_next=False)
    if out is None:
        out = torch.empty(B, OUT, dtype=torch.float32, device=draws.device)
    N.check_cuda(out, "out", torch.float32)
    if out.shape[0] < B or out.shape[1] != OUT:
        raise ValueError("out must be [B, 64]")
    nb = max(1, min(N.cu_count(draws.device) * 2, (B + 127) // 128))
    N.call("em_mlp_fused_forward", draws.data_ptr(), sidx.data_ptr() if sidx is not None else None, B, offset,
           img.data_ptr(), out.data_ptr(), nb, N.stream_handle(draws.device))
    return out


def adam_slab(slabs: torch.Tensor | None, nslab: int, grad_scale: float, params: torch.Tensor, m: torch.Tensor,
              v: torch.Tensor, hp: torch.Tensor, state: torch.Tensor, mode: int = 0, grad_io: torch.Tensor | None = None,
              img: torch.Tensor | None = None, loss_slabs: torch.Tensor | None = None,
              loss_out: torch.Tensor | None = None, loss_scale: float = 1.0, pre: bool = False) -> None:
    """mode 0: slab reduce + Adam; mode 1: slab reduce -> grad_io; mode 2: Adam from grad_io.
    ``pre``: the step counter ``state[0]`` was already advanced for this step
    (train_partials(step=state)), so no grid-wide ticket is drawn."""
    P = params.numel()
    stride = slabs.shape[1] if slabs is not None else P
    N.call("em_adam_slab", slabs.data_ptr() if slabs is not None else None, int(nslab), int(P), int(stride),
           float(grad_scale),
           params.data_ptr(), m.data_ptr(), v.data_ptr(), grad_io.data_ptr() if grad_io is not None else None,
           hp.data_ptr(), state.data_ptr(), int(mode) | (ADAM_PRE if pre else 0),
           img.data_ptr() if img is not None else None,
           loss_slabs.data_ptr() if loss_slabs is not None else None,
           loss_out.data_ptr() if loss_out is not None else None, float(loss_scale),
           N.stream_handle(params.device))


def adam_slab_xgmi(xgmi: int, slabs: torch.Tensor, nslab: int, grad_scale: float, params: torch.Tensor,
                   m: torch.Tensor, v: torch.Tensor, hp: torch.Tensor, state: torch.Tensor, loss_slabs: torch.Tensor,
                   img: torch.Tensor | None = None, loss_out: torch.Tensor | None = None, loss_scale: float = 1.0,
                   pre: bool = False, max_blocks: int = 0) -> None:
    """The DP optimizer step in ONE launch (csrc/adam.hip adam_slab_xgmi_kernel): this rank's slab
    reduction into its xGMI slot (block-sliced), the exchange, the rank-order sum of every rank's
    [grad | loss] and Adam.  ``max_blocks`` > 0 caps the grid (blocks loop over the slices)."""
    from ..parallel import xgmi as _xg  # noqa: F401  (registers the em_xgmi_* signatures)

    N.call("em_adam_slab_xgmi", xgmi, slabs.data_ptr(), int(nslab), int(slabs.shape[1]), float(grad_scale),
           params.numel(), params.data_ptr(), m.data_ptr(), v.data_ptr(), hp.data_ptr(), state.data_ptr(),
           img.data_ptr() if img is not None else None, loss_slabs.data_ptr(),
           loss_out.data_ptr() if loss_out is not None else None, float(loss_scale), int(pre), int(max_blocks),
           N.stream_handle(params.device))


def cast_bf16(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """fp32 -> bf16 (round to nearest even), one HIP launch (gradient buckets before a bf16 all-reduce)."""
    N.check_cuda(src, "src", torch.float32)
    N.check_cuda(dst, "dst", torch.bfloat16)
    if dst.numel() < src.numel():
        raise ValueError("dst too small")
    N.call("em_cast_f32_bf16", src.data_ptr(), dst.data_ptr(), src.numel(), N.stream_handle(src.device))
    return dst


def adam_flat(params: torch.Tensor, grad: torch.Tensor, m: torch.Tensor, v: torch.Tensor, hp: torch.Tensor,
              state: torch.Tensor, grad_scale: float = 1.0, shadow: torch.Tensor | None = None) -> None:
    """K6 over a flat fp32 buffer; ``grad`` fp32, or bf16 (a gradient all-reduced in bf16, widened in
    the kernel: moments and master weights stay fp32)."""
    for t, nm in ((params, "params"), (m, "m"), (v, "v")):
        N.check_cuda(t, nm, torch.float32)
    if shadow is not None:
        N.check_cuda(shadow, "shadow", torch.bfloat16)
    if grad.dtype == torch.bfloat16:
        N.check_cuda(grad, "grad", torch.bfloat16)
        N.call("em_adam_flat_bf16g", params.data_ptr(), grad.data_ptr(), m.data_ptr(), v.data_ptr(), params.numel(),
               hp.data_ptr(), state.data_ptr(), float(grad_scale),
               shadow.data_ptr() if shadow is not None else None, N.stream_handle(params.device))
        return
    N.check_cuda(grad, "grad", torch.float32)
    N.call("em_adam_flat", params.data_ptr(), grad.data_ptr(), m.data_ptr(), v.data_ptr(), params.numel(),
           hp.data_ptr(), state.data_ptr(), float(grad_scale), shadow.data_ptr() if shadow is not None else None,
           N.stream_handle(params.device))


METRIC_NAMES = ("loss", "acc", "acc_thr", "hits_main", "hits_star", "exact", "trivial_acc", "count")


def draw_metrics(logits: torch.Tensor, draws: torch.Tensor, B: int, loss: str = "softmax", offset: int = 0,
                 sidx: torch.Tensor | None = None) -> torch.Tensor:
    """Per-block partial sums [nblocks, 8] (see METRIC_NAMES); sum on the host in fp64."""
    _check_draws(draws, sidx, B, offset)
    N.check_cuda(logits, "logits", torch.float32)
    nb = (B + 255) // 256
    part = torch.zeros(max(nb, 1), 8, dtype=torch.float32, device=logits.device)
    N.call("em_draw_metrics", logits.data_ptr(), logits.stride(0), draws.data_ptr(),
           sidx.data_ptr() if sidx is not None else None, B, offset, LOSS_KINDS[loss], part.data_ptr(),
           N.stream_handle(logits.device))
    return part


def onehot_lags(draws: torch.Tensor, B: int, lags: int, offset: int = 0, sidx: torch.Tensor | None = None,
                out: torch.Tensor | None = None, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """K14 lag window: [B, 64 * lags] rows [onehot(draw i) | ... | onehot(draw i + lags - 1)] (each block
    62 live + 2 zero columns), i = sidx[s] or offset + s; the target of sample i is draw i + lags."""
    if lags < 1:
        raise ValueError("lags >= 1")
    if dtype not in (torch.bfloat16, torch.float32):
        raise ValueError("bf16 or fp32 output")
    _check_draws(draws[lags - 1:] if lags > 1 else draws, sidx, B, offset, need_next=False)
    if out is None:
        out = torch.empty(B, 64 * lags, dtype=dtype, device=draws.device)
    N.check_cuda(out, "out", dtype)
    if out.shape[0] < B or out.shape[1] != 64 * lags:
        raise ValueError(f"out must be [>= B, {64 * lags}]")
    N.call("em_onehot_lags", draws.data_ptr(), sidx.data_ptr() if sidx is not None else None, B, offset, lags,
           1 if dtype == torch.float32 else 0, out.data_ptr(), N.stream_handle(draws.device))
    return out


def onehot(draws: torch.Tensor, B: int, offset: int = 0, which: int = 0, bias: bool = False,
           sidx: torch.Tensor | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """K14: multi-hot bf16 [B, 64] of draws[idx + which] (which=1 -> targets)."""
    _check_draws(draws, sidx, B, offset, need_next=(which == 1))
    if out is None:
        out = torch.empty(B, 64, dtype=torch.bfloat16, device=draws.device)
    N.call("em_onehot_encode", draws.data_ptr(), sidx.data_ptr() if sidx is not None else None, B, offset, which,
           1 if bias else 0, out.data_ptr(), N.stream_handle(draws.device))
    return out
