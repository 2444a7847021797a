"""ctypes binding of libunsamflow_hip.so (C ABI: include/unsamflow_hip.h).

The library is the only compute path of this package: there is no CPU or
PyTorch fallback. If the library is missing or cannot be loaded, every op
raises ``RuntimeError`` (the product path fails loudly).

torch must be imported first so the library binds to the HIP runtime torch
already loaded (same SONAME ``libamdhip64.so.7``).
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch  # noqa: F401  (load torch's HIP runtime before the plugin)

_LIB_PATH = Path(os.environ.get("USF_LIB", Path(__file__).resolve().parent / "lib" / "libunsamflow_hip.so"))
ABI_VERSION = 8
PAD_ZEROS = 0
PAD_BORDER = 1

# exported symbols and their signatures; tests check the library exports all of them
_c_float_p = ctypes.c_void_p
_SIGNATURES = {
    "usf_abi_version": ([], ctypes.c_int),
    "usf_last_error_string": ([], ctypes.c_char_p),
    "usf_build_id": ([], ctypes.c_char_p),
    "usf_corr_fwd_f32": (
        [_c_float_p, _c_float_p, _c_float_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_corr_bwd_f32": (
        [_c_float_p] * 5 + [ctypes.c_int] * 5 + [ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_corr_fwd_ex_f32": (
        [_c_float_p] * 3 + [ctypes.c_longlong, ctypes.c_int, ctypes.c_float, ctypes.c_void_p, _c_float_p,
                             ctypes.c_longlong]
        + [ctypes.c_int] * 5 + [ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_corr_act_mask_words": ([ctypes.c_int] * 4, ctypes.c_longlong),
    "usf_corr_fwd_workspace": ([ctypes.c_int] * 5, ctypes.c_longlong),
    "usf_corr_bwd_ex_scratch": ([ctypes.c_int] * 5, ctypes.c_longlong),
    "usf_corr_bwd_ex_f32": (
        [_c_float_p] * 3 + [ctypes.c_longlong, _c_float_p, ctypes.c_void_p, ctypes.c_float] + [_c_float_p] * 3
        + [ctypes.c_int] * 5 + [ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_warp_fwd_f32": (
        [_c_float_p, _c_float_p, ctypes.c_longlong, _c_float_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_warp_fwd_up_f32": ([_c_float_p] * 4 + [ctypes.c_int] * 5 + [ctypes.c_void_p], ctypes.c_int),
    "usf_flow_upsample_bwd_sum_f32": ([_c_float_p] * 3 + [ctypes.c_int] * 5 + [ctypes.c_void_p], ctypes.c_int),
    "usf_warp_bwd_f32": (
        [_c_float_p, _c_float_p, ctypes.c_longlong, _c_float_p, _c_float_p, _c_float_p]
        + [ctypes.c_int] * 5
        + [ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_warp_bwd_ex_f32": (
        [_c_float_p, _c_float_p, ctypes.c_longlong, _c_float_p, _c_float_p, _c_float_p, ctypes.c_void_p,
         ctypes.c_longlong] + [ctypes.c_int] * 5 + [ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_warp_bwd_workspace": ([ctypes.c_int] * 3, ctypes.c_longlong),
    "usf_warp_bwd_persist_f32": (
        [_c_float_p, _c_float_p, ctypes.c_longlong, _c_float_p, _c_float_p, _c_float_p, ctypes.c_void_p,
         ctypes.c_longlong] + [ctypes.c_int] * 5 + [ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_warp_bwd_persist_workspace": ([ctypes.c_int] * 4, ctypes.c_longlong),
    "usf_occ_backward_persist_f32": (
        [_c_float_p, ctypes.c_longlong, _c_float_p, _c_float_p, ctypes.c_longlong] + [ctypes.c_int] * 3
        + [ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_occ_vis_pair_persist_f32": (
        [_c_float_p, ctypes.c_longlong, _c_float_p, _c_float_p, ctypes.c_longlong] + [ctypes.c_int] * 3
        + [ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_splat_map_f32": (
        [_c_float_p, ctypes.c_longlong, _c_float_p] + [ctypes.c_int] * 4 + [ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_occ_backward_f32": (
        [_c_float_p, ctypes.c_longlong, _c_float_p] + [ctypes.c_int] * 3 + [ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_occ_bidirection_f32": (
        [_c_float_p, ctypes.c_longlong, _c_float_p, ctypes.c_longlong, _c_float_p] + [ctypes.c_int] * 3
        + [ctypes.c_float, ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_photo_loss_partials": ([ctypes.c_int] * 3, ctypes.c_int),
    "usf_photo_loss_fwd_f32": (
        [_c_float_p] * 4 + [ctypes.c_longlong, _c_float_p, _c_float_p, _c_float_p] + [ctypes.c_int] * 5
        + [ctypes.c_float, ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_photo_loss_pair_fwd_f32": (
        [_c_float_p] * 5 + [ctypes.c_longlong, _c_float_p, _c_float_p, _c_float_p] + [ctypes.c_int] * 5
        + [ctypes.c_float, ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_photo_loss_pyramid_partials": ([ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int],
                                        ctypes.c_longlong),
    "usf_photo_loss_pyramid_fwd_f32": (
        [ctypes.c_int] + [ctypes.c_void_p] * 8 + [_c_float_p, ctypes.c_longlong, _c_float_p, ctypes.c_void_p]
        + [ctypes.c_int] * 3 + [ctypes.c_float, ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_photo_loss_pyramid_bwd_f32": (
        [ctypes.c_int, ctypes.c_void_p, _c_float_p, _c_float_p] + [ctypes.c_void_p] * 3 + [ctypes.c_int,
                                                                                            ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_photo_loss_bwd_f32": (
        [_c_float_p] * 4 + [ctypes.c_int] * 4 + [ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_flow_upsample_f32": ([_c_float_p] * 2 + [ctypes.c_int] * 5 + [ctypes.c_void_p], ctypes.c_int),
    "usf_flow_upsample_bwd_f32": ([_c_float_p] * 2 + [ctypes.c_int] * 5 + [ctypes.c_void_p], ctypes.c_int),
    "usf_convex_upsample_f32": (
        [_c_float_p] * 3 + [ctypes.c_int] * 4 + [ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_convex_upsample_bwd_scratch": ([ctypes.c_int] * 3, ctypes.c_longlong),
    "usf_convex_upsample_bwd_f32": (
        [_c_float_p] * 6 + [ctypes.c_int] * 4 + [ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_convex_upsample_pyramid_f32": (
        [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_convex_upsample_pyramid_bwd_scratch": ([ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int],
                                                ctypes.c_longlong),
    "usf_convex_upsample_pyramid_bwd_f32": (
        [ctypes.c_int] + [ctypes.c_void_p] * 5 + [_c_float_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "usf_area_pyramid_f32": ([_c_float_p] * 4 + [ctypes.c_int] * 4 + [ctypes.c_void_p], ctypes.c_int),
    "usf_set_variant": ([ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "usf_device_errors": ([ctypes.c_void_p, ctypes.c_int], ctypes.c_int),
    "usf_stream_copy_f32": ([_c_float_p, _c_float_p, ctypes.c_longlong, ctypes.c_void_p], ctypes.c_int),
}
EXPORTED_SYMBOLS = tuple(_SIGNATURES)

_lock = threading.Lock()
_lib = None
_load_error: str | None = None


def library_path() -> Path:
    return _LIB_PATH


def load() -> ctypes.CDLL:
    """Load (once) and return the plugin library; raise RuntimeError if absent."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not _LIB_PATH.exists():
            _load_error = (
                f"libunsamflow_hip.so not found at {_LIB_PATH}; build it with "
                "`python -m unsamflow_amd.build` (hipcc, gfx950)"
            )
            raise RuntimeError(_load_error)
        lib = ctypes.CDLL(str(_LIB_PATH), mode=ctypes.RTLD_LOCAL)
        for name, (argtypes, restype) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = restype
        v = lib.usf_abi_version()
        if v != ABI_VERSION:
            raise RuntimeError(f"libunsamflow_hip.so ABI version {v} != expected {ABI_VERSION}")
        _lib = lib
        return lib


def build_id() -> str:
    """The loaded library's build id (usf_build_id; unsamflow_amd.build.build_id)."""
    return load().usf_build_id().decode()


def is_available() -> bool:
    try:
        load()
        return True
    except (RuntimeError, OSError):
        return False


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().usf_last_error_string()
        msg = msg.decode() if msg else ""
        raise RuntimeError(f"{what} failed (rc={rc}): {msg}")


def stream_handle(device: torch.device) -> int:
    """hipStream_t of torch's current stream on ``device``."""
    return torch.cuda.current_stream(device).cuda_stream
