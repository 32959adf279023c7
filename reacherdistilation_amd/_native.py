"""ctypes binding of the in-tree native library libreacher.so (include/reacher.h,
include/reacher_distill.h).

There is no fallback: if the library is missing or fails to load, importing the product
raises.  torch is imported first so that libreacher.so binds to the HIP runtime torch
already loaded (both carry SONAME libamdhip64.so.7) and device pointers are shared.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL: shares torch's libamdhip64)

HERE = os.path.dirname(os.path.abspath(__file__))
# RD_LIB selects a diagnostic build (e.g. libreacher_stamps.so); default: the product library
LIB_PATH = os.path.join(HERE, os.environ.get("RD_LIB", "libreacher.so"))

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
F32 = ctypes.c_float
INT = ctypes.c_int

RD_RESET_PHILOX = 0
RD_RESET_TABLE = 1

# (name, restype, argtypes) for every symbol include/*.h declares
SIGNATURES = {
    # reacher.h
    "rd_create": (INT, [ctypes.POINTER(P), I64, I64, U64, INT, P]),
    "rd_destroy": (INT, [P]),
    "rd_set_stream": (INT, [P, P]),
    "rd_reset": (INT, [P, P]),
    "rd_step": (INT, [P, P, P, P, P]),
    "rd_set_state": (INT, [P, P, I32, I32]),
    "rd_get_state": (INT, [P, P, ctypes.POINTER(I32), ctypes.POINTER(I32)]),
    "rd_set_reset_mode": (INT, [P, INT, P, I32]),
    "rd_gym_reset_draws": (INT, [U64, I32, P]),
    "rd_crc32c": (ctypes.c_uint32, [P, I64, ctypes.c_uint32]),
    "rd_version": (ctypes.c_char_p, []),
    "rd_last_error": (ctypes.c_char_p, []),
    # reacher_comm.h
    "rd_comm_unique_id": (INT, [P]),
    "rd_comm_probe": (INT, [INT]),
    "rd_comm_create": (INT, [ctypes.POINTER(P), P, INT, INT, INT, ctypes.c_double]),
    "rd_comm_allreduce_f32": (INT, [P, P, I64, P]),
    "rd_comm_nranks": (INT, [P]),
    "rd_comm_query": (INT, [P, P, P, P, P]),
    "rd_comm_destroy": (INT, [P]),
    "rd_xcomm_create": (INT, [ctypes.POINTER(P), INT, INT, INT, I64, ctypes.c_double, P]),
    "rd_xcomm_connect": (INT, [P, P]),
    "rd_comm_check": (INT, [P]),
}

_lib = None


class NativeError(RuntimeError):
    pass


def load():
    """Load libreacher.so (build it in-tree first if the sources are newer and hipcc exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"{LIB_PATH} not found: build it with `python -m reacherdistilation_amd.build` "
            "(or __graft_entry__.build()).  There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue  # missing symbols are reported by exported_symbols()/tests
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols():
    lib = load()
    return {n: hasattr(lib, n) for n in SIGNATURES}


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = load().rd_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed (rc={rc}): {msg}")


def register(signatures: dict):
    """Add more symbol signatures (used by the distill binding)."""
    SIGNATURES.update(signatures)
    if _lib is not None:
        for name, (res, args) in signatures.items():
            fn = getattr(_lib, name, None)
            if fn is not None:
                fn.restype = res
                fn.argtypes = args


def ptr(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
