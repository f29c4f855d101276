"""ctypes binding to ``euromillioner_amd/lib/libem_native.so`` (our HIP/C++ code).

Loading rules (see ``_build.py``):
  * ``import torch`` happens first so the HIP runtime torch ships
    (SONAME ``libamdhip64.so.7``) is the one our library binds to.
  * On a machine with a GPU the library MUST load: every op raises
    ``NativeUnavailable`` instead of silently falling back to PyTorch.
  * ``EUROM_AUTOBUILD=1`` (default on) compiles the library when it is missing.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from .. import _build

_lock = threading.Lock()
_lib = None
_load_error: str | None = None


class NativeUnavailable(RuntimeError):
    pass


_c_void_p = ctypes.c_void_p
_i32 = ctypes.c_int
_i64 = ctypes.c_int64
_f32 = ctypes.c_float

# name -> (restype, argtypes)
_SIGS = {
    "em_mlp_fused_param_count": (_i32, []),
    "em_mlp_fused_image_bytes": (_i32, []),
    "em_mlp_fused_lds_bytes": (_i32, []),
    "em_mlp_fused_train": (_i32, [_c_void_p, _c_void_p, _i64, _i64, _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _c_void_p,
                                   _c_void_p]),
    "em_mlp_fused_train_f32": (_i32, [_c_void_p, _c_void_p, _i64, _i64, _c_void_p, _c_void_p, _c_void_p, _i32, _i32,
                                       _c_void_p, _c_void_p]),
    "em_mlp_fused_f32_lds_bytes": (_i32, []),
    "em_mlp_fused_forward": (_i32, [_c_void_p, _c_void_p, _i64, _i64, _c_void_p, _c_void_p, _i32, _c_void_p]),
    "em_mlp_fused_pack": (_i32, [_c_void_p, _c_void_p, _c_void_p]),
    "em_mlp_fused_slab_stride": (_i32, []),
    "em_adam_slab": (_i32, [_c_void_p, _i32, _i32, _i32, _f32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                            _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _f32, _c_void_p]),
    "em_adam_flat": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p, _f32, _c_void_p,
                            _c_void_p]),
    "em_adam_flat_bf16g": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p, _f32,
                                  _c_void_p, _c_void_p]),
    "em_cast_f32_bf16": (_i32, [_c_void_p, _c_void_p, _i64, _c_void_p]),
    "em_draw_metrics": (_i32, [_c_void_p, _i32, _c_void_p, _c_void_p, _i64, _i64, _i32, _c_void_p, _c_void_p]),
    "em_onehot_encode": (_i32, [_c_void_p, _c_void_p, _i64, _i64, _i32, _i32, _c_void_p, _c_void_p]),
    "em_onehot_lags": (_i32, [_c_void_p, _c_void_p, _i64, _i64, _i32, _i32, _c_void_p, _c_void_p]),
    "em_rows_to_masks": (_i32, [_c_void_p, _i64, _c_void_p, _c_void_p]),
    "em_gen_masks": (_i32, [ctypes.c_uint64, ctypes.c_uint32, _i64, _i64, _c_void_p, _c_void_p, _c_void_p]),
    "em_gen_masks_at": (_i32, [ctypes.c_uint64, ctypes.c_uint32, _i64, _i64, _i64, _c_void_p, _c_void_p, _c_void_p]),
}


def _register(lib):
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue  # optional (older build); `call` raises if used
        fn.restype = res
        fn.argtypes = args


def register_signatures(sigs: dict):
    """Extension point: other op modules add their C-ABI signatures here."""
    _SIGS.update(sigs)
    if _lib is not None:
        _register(_lib)


def lib():
    """Return the loaded library (building it if needed)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = os.environ.get("EUROM_NATIVE_LIB") or _build.lib_path()  # override: A/B builds
        try:
            if not os.path.exists(path) or os.environ.get("EUROM_FORCE_BUILD") == "1":
                if os.environ.get("EUROM_AUTOBUILD", "1") != "1":
                    raise NativeUnavailable(f"{path} missing and EUROM_AUTOBUILD=0")
                _build.build()
            handle = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            _register(handle)
            _lib = handle
        except Exception as e:  # noqa: BLE001
            _load_error = f"{type(e).__name__}: {e}"
            raise NativeUnavailable(f"native library unavailable: {_load_error}") from e
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except NativeUnavailable:
        return False


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def call(name: str, *args) -> None:
    fn = getattr(lib(), name, None)
    if fn is None:
        raise NativeUnavailable(f"symbol {name} missing from {_build.lib_path()} (rebuild)")
    rc = fn(*args)
    if rc != 0:
        if rc == -1:
            raise ValueError(f"{name}: invalid arguments")
        raise RuntimeError(f"{name}: HIP error {rc}")


def query(name: str, *args):
    """Call a native function whose return value is data (a size, a count), not a status code."""
    fn = getattr(lib(), name, None)
    if fn is None:
        raise NativeUnavailable(f"symbol {name} missing from {_build.lib_path()} (rebuild)")
    return fn(*args)


def cu_count(device: torch.device | int | None = None) -> int:
    return torch.cuda.get_device_properties(device if device is not None else torch.cuda.current_device()).multi_processor_count


def check_cuda(t: torch.Tensor, name: str, dtype=None, contiguous=True):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if contiguous and not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
