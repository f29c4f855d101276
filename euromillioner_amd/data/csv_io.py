"""CSV materialisation and loading (reference layer L4 + the DMatrix CSV loader X1).

Reference behaviour (``Main.java:69-111``):
* header ``"day_of_week, month, day, year, first, second, third, fourth, fift,; special_1, special_2,"``
  (typos, stray ``;``, trailing comma, no newline) written to two temp files;
* each record is 11 fields each followed by ``", "`` and **no record terminator**
  (defect D-b: each file is one physical line);
* rows with index < int(0.7 n) go to the train file, the rest to validation;
* ``new DMatrix(path + "?format=csv&label_column=0")`` parses them (header as data: D-c).

Here:
* :func:`write_draws_csv` / :func:`read_draws_csv` — proper newline-terminated CSV
  with an explicit header (the fixed format);
* :func:`write_reference_csv` / :func:`read_reference_csv` — byte-compatible with the
  reference's quirky output, for parity demonstrations;
* :func:`load_numeric_csv` — the native multithreaded loader (``csrc/host/csv_loader.cpp``)
  with ``label_column`` semantics like dmlc's ``?format=csv&label_column=k``.
"""
from __future__ import annotations

import csv
import ctypes
import datetime as _dt
import os

import numpy as np

from .draws import REFERENCE_COLUMNS, DrawSet, featurize_raw, positional_split

REFERENCE_HEADER = "day_of_week, month, day, year, first, second, third, fourth, fift,; special_1, special_2,"
OUR_HEADER = ["date"] + REFERENCE_COLUMNS


def write_draws_csv(path: str, ds: DrawSet) -> None:
    raw = featurize_raw(ds) if ds.dates is not None else None
    with open(path, "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(OUR_HEADER)
        for i in range(len(ds)):
            if raw is not None:
                date = str(ds.dates[i])
                row = [date] + [int(v) for v in raw[i]]
            else:
                row = ["", 0, 0, 0, 0] + [int(v) for v in ds.numbers[i, :7]]
            w.writerow(row)


def read_draws_csv(path: str, header: bool | None = None) -> DrawSet:
    """Our CSV (with ``date`` column), the reference's 11 columns with a header, or headerless 11/12 cols.
    ``header``: None = detect, True/False = force (``--header yes|no``)."""
    with open(path, newline="", encoding="utf-8") as f:
        rows = [r for r in csv.reader(f) if any(c.strip() for c in r)]
    if not rows:
        return DrawSet(np.zeros((0, 8), np.uint8))
    head = [c.strip().lower() for c in rows[0]]

    def numeric(c: str) -> bool:
        try:
            float(c)
            return True
        except ValueError:
            return False

    has_header = (not all(numeric(c) for c in head if c) or "date" in head) if header is None else bool(header)
    body = rows[1:] if has_header else rows
    nums, dates = [], []
    for r in body:
        r = [c.strip() for c in r]
        while r and r[-1] == "":
            r.pop()
        if has_header and "date" in head:
            d = r[head.index("date")]
            vals = [int(float(c)) for c in r[head.index("date") + 1:]]
            dates.append(np.datetime64(d, "D") if d else np.datetime64("NaT"))
        else:
            vals = [int(float(c)) for c in r]
            if len(vals) >= 11:
                dow, m, d, y = vals[:4]
                dates.append(np.datetime64(_dt.date(y, m, d), "D") if y > 0 else np.datetime64("NaT"))
            else:
                dates.append(np.datetime64("NaT"))
        n7 = vals[-7:]
        nums.append(n7 + [0])
    arr = np.array(nums, dtype=np.uint8).reshape(-1, 8)
    dd = np.array(dates, dtype="datetime64[D]")
    return DrawSet(arr, None if np.isnat(dd).all() else dd, {"source": "csv", "path": path})


def write_reference_csv(train_path: str, val_path: str, ds: DrawSet, train_pct: float = 70.0) -> int:
    """Reproduce the reference's two CSV files byte-for-byte (Main.java:69-108).  Returns the margin."""
    raw = featurize_raw(ds)
    margin = positional_split(len(ds), train_pct)
    with open(train_path, "a", encoding="utf-8") as ft, open(val_path, "a", encoding="utf-8") as fv:
        ft.write(REFERENCE_HEADER)
        fv.write(REFERENCE_HEADER)
        for i in range(len(ds)):
            rec = "".join(f"{int(v)}, " for v in raw[i])
            (ft if i < margin else fv).write(rec)
    return margin


def read_reference_csv(path: str) -> np.ndarray:
    """Parse the reference's one-line CSV: numeric tokens regrouped into 11-field records."""
    with open(path, encoding="utf-8") as f:
        text = f.read()
    toks = []
    for t in text.replace(";", ",").replace("\n", ",").split(","):
        t = t.strip()
        if not t:
            continue
        try:
            toks.append(int(float(t)))
        except ValueError:
            continue  # header words
    if len(toks) % 11:
        raise ValueError(f"{path}: {len(toks)} numeric fields is not a multiple of 11")
    return np.array(toks, dtype=np.int64).reshape(-1, 11)


def reference_records_to_drawset(rec: np.ndarray) -> DrawSet:
    dates = np.array([np.datetime64(_dt.date(int(y), int(m), int(d)), "D") for _, m, d, y in rec[:, :4]],
                     dtype="datetime64[D]")
    nums = np.zeros((len(rec), 8), np.uint8)
    nums[:, :7] = rec[:, 4:11]
    return DrawSet(nums, dates, {"source": "reference-csv"})


def load_numeric_csv(path: str, skip_header: bool = True, label_column: int | None = 0, nthreads: int = 0):
    """Native CSV -> (X float32 [n, d], y float32 [n] or None).  NaN marks non-numeric/missing fields."""
    from ..utils import hostlib

    h = hostlib.lib()
    ncols = ctypes.c_int64(0)
    n = h.emh_csv_shape(path.encode(), 1 if skip_header else 0, ctypes.byref(ncols))
    if n < 0:
        raise FileNotFoundError(path)
    d = int(ncols.value)
    out = np.empty((n, d), dtype=np.float32)
    if n:
        rc = h.emh_csv_load(path.encode(), 1 if skip_header else 0, n, d, out.ctypes.data,
                            int(nthreads or min(8, os.cpu_count() or 1)))
        if rc != 0:
            raise RuntimeError(f"emh_csv_load failed ({rc})")
    if label_column is None:
        return out, None
    if not 0 <= label_column < d:
        raise ValueError(f"label_column {label_column} out of range for {d} columns")
    y = out[:, label_column].copy()
    X = np.delete(out, label_column, axis=1)
    return X, y


def load_numeric_csv_tensor(path: str, skip_header: bool = True, label_column: int | None = 0, pin: bool = True):
    """X1: native CSV -> torch tensors in pinned (page-locked) host memory when a GPU is present,
    ready for an async ``.to(device, non_blocking=True)`` upload."""
    import torch

    X, y = load_numeric_csv(path, skip_header, label_column)
    pin = pin and torch.cuda.is_available()
    tx = torch.from_numpy(X)
    ty = torch.from_numpy(y) if y is not None else None
    if pin:
        tx = tx.pin_memory()
        ty = ty.pin_memory() if ty is not None else None
    return tx, ty
