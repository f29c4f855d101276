"""Draw containers, featurizers and the positional train/validation split.

Row layout everywhere (host numpy and device tensors): ``uint8[8]`` =
5 main numbers (1..50), 2 stars (1..12), 1 zero pad — 8 bytes so the GPU reads a
row with one ``uint2`` load.  A *sample* ``i`` is the pair (draw i -> draw i+1):
input = multi-hot of draw ``i``, target = multi-hot of draw ``i+1`` (SURVEY.md
§2.4 N2).

Reference parity:
* ``featurize_raw`` = the reference's per-row CSV record (``Main.java:86-102``):
  ``dayOfWeek (ISO 1-7), month, day, year`` from the date, then the numbers
  verbatim — 11 integers, label column 0 (``Main.java:110-111``).
* ``positional_split`` = ``(int)(0.70 * rows)`` with ``i < margin`` -> train
  (``Main.java:83-84,103-104``).
"""
from __future__ import annotations

import dataclasses

import numpy as np

N_MAIN, N_STAR = 50, 12
N_OUT = N_MAIN + N_STAR  # 62
REFERENCE_COLUMNS = ["day_of_week", "month", "day", "year", "first", "second", "third", "fourth", "fifth",
                     "special_1", "special_2"]


@dataclasses.dataclass
class DrawSet:
    numbers: np.ndarray  # [N, 8] uint8
    dates: np.ndarray | None = None  # [N] datetime64[D]
    meta: dict = dataclasses.field(default_factory=dict)

    def __post_init__(self):
        self.numbers = np.ascontiguousarray(self.numbers, dtype=np.uint8)
        if self.numbers.ndim != 2 or self.numbers.shape[1] != 8:
            raise ValueError(f"numbers must be [N, 8] uint8, got {self.numbers.shape}")
        if self.dates is not None and len(self.dates) != len(self.numbers):
            raise ValueError("dates/numbers length mismatch")

    def __len__(self) -> int:
        return len(self.numbers)

    @property
    def n_samples(self) -> int:
        return max(0, len(self) - 1)

    def validate(self) -> None:
        m, s = self.numbers[:, :5].astype(int), self.numbers[:, 5:7].astype(int)
        if (m < 1).any() or (m > 50).any():
            raise ValueError("main numbers must be in 1..50")
        if (s < 1).any() or (s > 12).any():
            raise ValueError("stars must be in 1..12")
        if (np.sort(m, 1)[:, 1:] == np.sort(m, 1)[:, :-1]).any() or (s[:, 0] == s[:, 1]).any():
            raise ValueError("numbers within a draw must be distinct")

    def slice(self, a: int, b: int) -> "DrawSet":
        return DrawSet(self.numbers[a:b], None if self.dates is None else self.dates[a:b], dict(self.meta))

    @staticmethod
    def synthetic(n: int | None = None, seed: int = 0, planted: float = 0.0, calendar: bool = True) -> "DrawSet":
        """``n=None`` -> exactly the reference's date range (2004-02-13..2020-06-14, ~1.33k draws)."""
        from . import synthetic as syn

        if n is None:
            dates = syn.draw_dates()
        elif calendar and n <= 200_000:
            dates = syn.draw_dates(n=n)
        elif calendar:
            dates = syn.draw_dates_fast(n)
        else:
            dates = None
        nn = len(dates) if dates is not None else int(n)
        sm = syn.star_max_for(dates) if dates is not None else None
        nums, perm = syn.generate_draws(nn, seed=seed, planted=planted, star_max=sm)
        return DrawSet(nums, dates, {"source": "synthetic", "seed": seed, "planted": planted, "perm": perm})


def mask_bits(numbers: np.ndarray) -> np.ndarray:
    """[N, 8] rows -> [N] uint64 feature masks (bit n-1 for main n, bit 49+s for star s)."""
    nums = numbers.astype(np.int64)
    m = np.zeros(len(numbers), dtype=np.uint64)
    for k in range(7):
        v = nums[:, k]
        if k < 5:
            ok, bit = (v >= 1) & (v <= 50), v - 1
        else:
            ok, bit = (v >= 1) & (v <= 12), v + 49
        sh = np.left_shift(np.uint64(1), np.where(ok, bit, 0).astype(np.uint64))
        m |= np.where(ok, sh, np.uint64(0))
    return m


def multi_hot(numbers: np.ndarray, width: int = N_OUT, bias: bool = False) -> np.ndarray:
    """[N, 8] draw rows -> [N, width] float32 multi-hot (7 ones; optional bias column 62)."""
    n = len(numbers)
    out = np.zeros((n, width), dtype=np.float32)
    rows = np.arange(n)
    for k in range(5):
        v = numbers[:, k].astype(np.int64)
        ok = (v >= 1) & (v <= 50)
        out[rows[ok], v[ok] - 1] = 1.0
    for k in (5, 6):
        v = numbers[:, k].astype(np.int64)
        ok = (v >= 1) & (v <= 12)
        out[rows[ok], 49 + v[ok]] = 1.0
    if bias:
        if width <= 62:
            raise ValueError("bias column needs width >= 63")
        out[:, 62] = 1.0
    return out


def lag_features(numbers: np.ndarray, lags: int = 1) -> tuple[np.ndarray, np.ndarray]:
    """Sliding window: input = multi-hot of draws t-lags+1..t (62*lags), target = draw t+1."""
    mh = multi_hot(numbers)
    n = len(numbers)
    if n <= lags:
        return np.zeros((0, 62 * lags), np.float32), np.zeros((0, 62), np.float32)
    X = np.concatenate([mh[k:n - lags + k] for k in range(lags)], axis=1)
    Y = mh[lags:]
    return X, Y


def featurize_raw(ds: DrawSet) -> np.ndarray:
    """The reference's 11 integer columns (Main.java:91-101): dow, month, day, year, n1..n5, s1, s2."""
    if ds.dates is None:
        raise ValueError("raw featurization needs draw dates")
    d = ds.dates.astype("datetime64[D]")
    y = d.astype("datetime64[Y]").astype(int) + 1970
    mo = d.astype("datetime64[M]").astype(int) % 12 + 1
    day = (d - d.astype("datetime64[M]")).astype(int) + 1
    dow = (d.astype("int64") + 3) % 7 + 1  # ISO: Monday=1 .. Sunday=7 (1970-01-01 = Thursday = 4)
    return np.column_stack([dow, mo, day, y, ds.numbers[:, :7].astype(np.int64)]).astype(np.int64)


def positional_split(n: int, train_pct: float = 70.0) -> int:
    """Index margin: rows with i < margin train, the rest validate (Main.java:83-84)."""
    return int((train_pct / 100.0) * n)
