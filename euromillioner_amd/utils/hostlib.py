"""ctypes binding to ``libem_host.so`` — pure C++ host code (no GPU needed).

Holds the native data-path pieces: the synthetic draw generator
(``csrc/host/datagen.cpp``) and the multithreaded CSV loader
(``csrc/host/csv_loader.cpp``, the X1 / dmlc-core CSV equivalent of
``Main.java:110-111``).
"""
from __future__ import annotations

import ctypes
import os
import threading

from .. import _build

_lock = threading.Lock()
_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            path = _build.host_lib_path()
            if not os.path.exists(path) or os.environ.get("EUROM_FORCE_BUILD") == "1":
                _build.build_host()
            h = ctypes.CDLL(path)
            h.emh_generate_draws.restype = ctypes.c_int
            h.emh_generate_draws.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p]
            h.emh_csv_shape.restype = ctypes.c_int64
            h.emh_csv_shape.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
            h.emh_csv_load.restype = ctypes.c_int
            h.emh_csv_load.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                       ctypes.c_int]
            _lib = h
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except Exception:  # noqa: BLE001
        return False
