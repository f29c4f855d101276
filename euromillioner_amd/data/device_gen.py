"""HBM-resident synthetic datasets: draws generated on the GPU, straight into feature masks.

The north star sizes the small-MLP's data for MI355X's 288 GB of HBM (BASELINE.json "Mini-batches
... tiled to fill 288 GB of HBM per GPU").  The host generator
(``synthetic.generate_draws``, one splitmix64 stream) produces ~10^8 draws/s and would need minutes,
plus host RAM, for tens of billions of draws.  Here the sequence is cut into independent segments of
``seg_len`` draws.  One GPU thread generates each segment, and it writes the 8-byte masks that the
trainers consume (bit n-1: main number n, bit 49+s: star s; see ``ops.fused_mlp.rows_to_masks``).
Filling HBM is then bounded by HBM write bandwidth, not by the host.

The rules per segment match ``synthetic.generate_draws_py``: 5 distinct mains in 1..50, 2 distinct
stars in 1..12, and an optional planted Markov map.  Under that map, each main/star of draw t-1
maps through a fixed permutation into draw t with probability ``planted``.  Both permutations come
from the host generator's stream for the same seed, so the planted structure matches
``generate_draws``.  The first draw of every segment is unplanted.  The RNG calls are cheaper than the
sequential spec's: Lemire ranges, and 24-bit thresholds for the planted coin.
:func:`generate_masks_py` below is the specification that the HIP kernel (``csrc/datagen.hip``)
reproduces bit for bit."""
from __future__ import annotations

import numpy as np
import torch

from .synthetic import _perm, _SplitMix64

M64 = (1 << 64) - 1
SEG_SALT = 0xD1B54A32D192ED03


def _seg_seed(seed: int, seg: int) -> int:
    """Segment stream seed: the splitmix64 finaliser of seed ^ (seg + 1) * salt."""
    z = (seed ^ (((seg + 1) * SEG_SALT) & M64)) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def permutations(seed: int) -> np.ndarray:
    """The planted maps [pim(50) | pis(12)] as 1-based values (same as ``generate_draws``'s perm)."""
    g = _SplitMix64(seed)
    return np.array(_perm(g, 50) + _perm(g, 12), dtype=np.int32)


def planted_threshold(planted: float) -> int:
    if not 0.0 <= planted <= 1.0:
        raise ValueError("planted must be in [0, 1]")
    return int(round(planted * (1 << 24)))


def _check_first(first: int, seg_len: int) -> int:
    if first < 0 or first % seg_len:
        raise ValueError(f"first ({first}) must be a non-negative multiple of seg_len ({seg_len})")
    return first // seg_len


def generate_masks_py(n: int, seed: int = 0, planted: float = 0.0, seg_len: int = 4096, first: int = 0) -> np.ndarray:
    """Specification: draws [first, first + n) of the sequence as masks [n] int64 (slow; for tests and
    small n).  ``first`` must be a multiple of ``seg_len`` (a shard starts on a segment boundary)."""
    seg0 = _check_first(first, seg_len)
    perm = permutations(seed)
    pim, pis = perm[:50], perm[50:]
    thr = planted_threshold(planted)
    out = np.zeros(n, dtype=np.uint64)
    for seg in range((n + seg_len - 1) // seg_len):
        g = _SplitMix64(_seg_seed(seed, seg0 + seg))

        def rng_range(k: int) -> int:
            return ((g.next() >> 32) * k) >> 32

        prev = 0
        for t in range(seg * seg_len, min(n, (seg + 1) * seg_len)):
            mask = 0
            if t > seg * seg_len and thr > 0:
                for k in range(50):  # previous mains in ascending order
                    if (prev >> k) & 1:
                        if (g.next() >> 40) < thr:
                            mask |= 1 << (int(pim[k]) - 1)
            while bin(mask & ((1 << 50) - 1)).count("1") < 5:
                mask |= 1 << rng_range(50)
            if t > seg * seg_len and thr > 0:
                for k in range(12):
                    if (prev >> (50 + k)) & 1:
                        if (g.next() >> 40) < thr:
                            mask |= 1 << (49 + int(pis[k]))
            while bin(mask >> 50).count("1") < 2:
                mask |= 1 << (50 + rng_range(12))
            out[t] = mask
            prev = mask
    return out.view(np.int64)


def generate_masks(n: int, seed: int = 0, planted: float = 0.0, seg_len: int = 4096,
                   device: torch.device | str = "cuda", out: torch.Tensor | None = None, first: int = 0) -> torch.Tensor:
    """Draws [first, first + n) of the sequence as masks [n] int64 generated on the GPU
    (``em_gen_masks_at``), HBM-resident.  Every rank of a data-parallel job passes the same seed
    (same planted maps = same task) and its own ``first`` (a disjoint shard of one sequence)."""
    seg0 = _check_first(first, seg_len)
    from ..ops import _native as N

    if n <= 0 or seg_len <= 0:
        raise ValueError("n and seg_len must be positive")
    dev = torch.device(device)
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=dev)
    elif out.dtype != torch.int64 or out.numel() < n or not out.is_contiguous():
        raise ValueError("out must be a contiguous int64 tensor with >= n elements")
    perm = torch.from_numpy(permutations(seed)).to(dev)
    N.call("em_gen_masks_at", seed & M64, planted_threshold(planted), n, seg_len, seg0, perm.data_ptr(),
           out.data_ptr(), N.stream_handle(dev))
    return out[:n]


def gb_to_draws(gb: float) -> int:
    """Number of 8-byte draw masks in ``gb`` GiB."""
    return int(gb * (1 << 30)) // 8


def region(a: int, b: int, seg_len: int = 4096) -> tuple[int, int, int]:
    """Segment-aligned cover of draws [a, b): (first, n, skip) with first % seg_len == 0 and
    draws [a, b) == generated[skip : skip + b - a]."""
    if not 0 <= a <= b:
        raise ValueError("need 0 <= a <= b")
    first = (a // seg_len) * seg_len
    return first, max(b - first, 1), a - first
