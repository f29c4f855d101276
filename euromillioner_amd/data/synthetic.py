"""Euromillions calendar + seeded synthetic draw generator.

Replaces the reference's acquisition stage — an HTTP GET of the portalseven.com
results table for 1900-01-01..2020-06-14 (``Main.java:37-58``) — because there is
no network.  Domain rules reproduced:

* main numbers: 5 distinct values 1..50;
* stars: 2 distinct values 1..9 before 2011-05-10, 1..11 until 2016-09-23,
  1..12 from 2016-09-27;
* draws on Fridays from 2004-02-13, Tuesdays and Fridays from 2011-05-10.

``generate_draws`` optionally plants a learnable Markov structure (see
``csrc/host/datagen.cpp``).  The pure-Python implementation here is the
specification; the C++ one (same splitmix64 stream, same call order) is used for
large ``n`` and is tested bit-for-bit against it.
"""
from __future__ import annotations

import ctypes
import datetime as _dt

import numpy as np

FIRST_DRAW = _dt.date(2004, 2, 13)
TUESDAYS_FROM = _dt.date(2011, 5, 10)
STARS_11_FROM = _dt.date(2011, 5, 10)
STARS_12_FROM = _dt.date(2016, 9, 24)  # first 12-star draw was 2016-09-27
REFERENCE_TO = _dt.date(2020, 6, 14)  # Main.java:37 toDate


def draw_dates(start: _dt.date = FIRST_DRAW, end: _dt.date | None = REFERENCE_TO, n: int | None = None) -> np.ndarray:
    """Draw dates following the schedule; either up to ``end`` or exactly ``n`` dates."""
    out = []
    d = start
    while True:
        if n is not None and len(out) >= n:
            break
        if n is None and end is not None and d > end:
            break
        wd = d.weekday()  # Mon=0 .. Fri=4
        if wd == 4 or (wd == 1 and d >= TUESDAYS_FROM):
            out.append(d)
        d += _dt.timedelta(days=1)
    return np.array(out, dtype="datetime64[D]")


def draw_dates_fast(n: int, start: _dt.date = FIRST_DRAW) -> np.ndarray:
    """Vectorised schedule for very long synthetic sequences (same result as ``draw_dates(n=n)``)."""
    est_days = int(n * 7 / 2) + 4000
    days = np.arange(np.datetime64(start, "D"), np.datetime64(start, "D") + est_days)
    wd = (days.astype("int64") + 3) % 7  # 1970-01-01 was a Thursday (=3 with Mon=0)
    keep = (wd == 4) | ((wd == 1) & (days >= np.datetime64(TUESDAYS_FROM, "D")))
    out = days[keep]
    if len(out) < n:
        raise RuntimeError("date estimate too small")
    return out[:n]


def star_max_for(dates: np.ndarray) -> np.ndarray:
    d = dates.astype("datetime64[D]")
    out = np.full(d.shape, 12, dtype=np.int32)
    out[d < np.datetime64(STARS_12_FROM, "D")] = 11
    out[d < np.datetime64(STARS_11_FROM, "D")] = 9
    return out


class _SplitMix64:
    M = (1 << 64) - 1

    def __init__(self, seed: int):
        self.s = seed & self.M

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & self.M
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & self.M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & self.M
        return z ^ (z >> 31)

    def uint(self, n: int) -> int:
        return self.next() % n

    def u01(self) -> float:
        return (self.next() >> 11) * (1.0 / 9007199254740992.0)


def _perm(g: _SplitMix64, n: int) -> list[int]:
    a = list(range(1, n + 1))
    for i in range(n - 1, 0, -1):
        j = g.uint(i + 1)
        a[i], a[j] = a[j], a[i]
    return a


def generate_draws_py(n: int, seed: int = 0, planted: float = 0.0, star_max: np.ndarray | None = None):
    """Reference (specification) implementation.  Returns (draws[n,8] uint8, perm[62] int32)."""
    if not 0.0 <= planted <= 1.0:
        raise ValueError("planted must be in [0, 1]")
    g = _SplitMix64(seed)
    pim = _perm(g, 50)
    pis = _perm(g, 12)
    out = np.zeros((n, 8), dtype=np.uint8)
    pm: list[int] = []
    ps: list[int] = []
    for t in range(n):
        smax = int(star_max[t]) if star_max is not None else 12
        m: list[int] = []
        if t > 0 and planted > 0.0:
            for k in range(5):
                if g.u01() < planted:
                    c = pim[pm[k] - 1]
                    if c not in m:
                        m.append(c)
        while len(m) < 5:
            c = 1 + g.uint(50)
            if c not in m:
                m.append(c)
        s: list[int] = []
        if t > 0 and planted > 0.0:
            for k in range(2):
                if g.u01() < planted:
                    c = pis[ps[k] - 1]
                    if c <= smax and c not in s:
                        s.append(c)
        while len(s) < 2:
            c = 1 + g.uint(smax)
            if c not in s:
                s.append(c)
        m.sort()
        s.sort()
        out[t, :5] = m
        out[t, 5:7] = s
        pm, ps = m, s
    return out, np.array(pim + pis, dtype=np.int32)


def generate_draws(n: int, seed: int = 0, planted: float = 0.0, star_max: np.ndarray | None = None,
                   native: bool | None = None):
    """Generate ``n`` draws; uses the C++ generator when available (identical output)."""
    if native is None:
        native = n > 2000
    if native:
        from ..utils import hostlib

        try:
            h = hostlib.lib()
        except Exception:  # noqa: BLE001
            h = None
        if h is not None:
            out = np.zeros((n, 8), dtype=np.uint8)
            perm = np.zeros(62, dtype=np.int32)
            sm = None
            if star_max is not None:
                sm = np.ascontiguousarray(star_max, dtype=np.int32)
                if sm.shape != (n,):
                    raise ValueError("star_max must have shape [n]")
            rc = h.emh_generate_draws(ctypes.c_uint64(seed & ((1 << 64) - 1)), n, float(planted),
                                      sm.ctypes.data if sm is not None else None, out.ctypes.data, perm.ctypes.data)
            if rc != 0:
                raise ValueError(f"emh_generate_draws failed ({rc})")
            return out, perm
    return generate_draws_py(n, seed, planted, star_max)
