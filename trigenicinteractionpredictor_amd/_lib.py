"""ctypes binding of libmmsbm.so (include/mmsbm.h).

There is no CPU fallback: if the shared object is missing or does not load,
every engine call raises.  torch is imported first on purpose: the library is
linked against libamdhip64.so.7, and loading it after torch makes the dynamic
linker reuse torch's HIP runtime (same SONAME) instead of a second copy, so
device pointers from torch tensors are valid in our kernels.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

from .build import LIB

MMSBM_OK = 0
MMSBM_ERR_INVALID = -1
MMSBM_ERR_HIP = -2
MMSBM_ERR_ZERO_DEGREE = -3
MMSBM_ERR_UNSUPPORTED = -4
SET_TRAIN = 0
SET_TEST = 1
FAMILY_AUTO = 0     # mmsbm_set_family: the small-K kernel family from B
FAMILY_SKU = 1      # the three-stream fused E-step
FAMILY_SKY = 2      # the stream-0 E-step with Y entries
CHUNK = 4
MAX_K = 32

# exported symbol -> (restype, argtypes); mirrors include/mmsbm.h
_c_int, _c_i32, _c_i64, _c_dbl, _vp = ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
SIGNATURES = {
    "mmsbm_version": (_c_int, []),
    "mmsbm_chunk": (_c_int, []),
    "mmsbm_build_id": (ctypes.c_char_p, []),
    "mmsbm_last_error": (ctypes.c_char_p, []),
    "mmsbm_create": (_c_int, [_c_int, ctypes.POINTER(_vp)]),
    "mmsbm_destroy": (_c_int, [_vp]),
    "mmsbm_set_shape": (_c_int, [_vp, _c_i32, _c_i32, _c_i32, _c_i32, _c_dbl]),
    "mmsbm_set_links": (_c_int, [_vp, _c_i32, _vp, _vp, _c_i64]),
    "mmsbm_set_degree": (_c_int, [_vp, _vp]),
    "mmsbm_workspace_bytes": (_c_int, [_vp, ctypes.POINTER(_c_i64)]),
    "mmsbm_set_workspace": (_c_int, [_vp, _vp, _c_i64]),
    "mmsbm_iterate": (_c_int, [_vp, _vp, _vp, _c_i32, _vp]),
    "mmsbm_loglik": (_c_int, [_vp, _c_i32, _vp, _vp, _vp, _vp]),
    "mmsbm_predict": (_c_int, [_vp, _vp, _c_i64, _vp, _vp, _vp, _vp]),
    "mmsbm_accumulate": (_c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "mmsbm_mstep": (_c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "mmsbm_plan_info": (_c_int, [_vp, _c_i32, ctypes.POINTER(_c_i64)]),
    "mmsbm_set_theta_addend": (_c_int, [_vp, _vp]),
    "mmsbm_set_family": (_c_int, [_vp, _c_i32]),
    "mmsbm_set_active": (_c_int, [_vp, _c_i32]),
    "mmsbm_timing": (_c_int, [_vp, _c_i32]),
    "mmsbm_timing_result": (_c_int, [_vp, _c_i32, ctypes.POINTER(_c_dbl), ctypes.POINTER(_c_i64)]),
    "mmsbm_time_kernel": (_c_int, [_vp, _c_i32, _vp, _vp, _c_i32, _vp, ctypes.POINTER(_c_dbl)]),
    # include/mmsbm_pairs.h — the joint model's pair lattice
    "mmsbm_pairs_create": (_c_int, [_c_int, ctypes.POINTER(_vp)]),
    "mmsbm_pairs_destroy": (_c_int, [_vp]),
    "mmsbm_pairs_set_shape": (_c_int, [_vp, _c_i32, _c_i32, _c_i32, _c_i32, _c_dbl]),
    "mmsbm_pairs_set_links": (_c_int, [_vp, _c_i32, _vp, _vp, _c_i64]),
    "mmsbm_pairs_workspace_bytes": (_c_int, [_vp, ctypes.POINTER(_c_i64)]),
    "mmsbm_pairs_set_workspace": (_c_int, [_vp, _vp, _c_i64]),
    "mmsbm_pairs_accumulate": (_c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "mmsbm_joint_iterate": (_c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _c_i32, _vp]),
    "mmsbm_pairs_qstep": (_c_int, [_vp, _vp, _vp, _vp]),
    "mmsbm_pairs_loglik": (_c_int, [_vp, _c_i32, _vp, _vp, _vp, _vp]),
    "mmsbm_pairs_predict": (_c_int, [_vp, _vp, _c_i64, _vp, _vp, _vp, _vp]),
    "mmsbm_pairs_plan_info": (_c_int, [_vp, _c_i32, ctypes.POINTER(_c_i64)]),
}

_lib = None


class MMSBMError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("mmsbm error %d: %s" % (code, msg))
        self.code = code


def load(path: str = LIB) -> ctypes.CDLL:
    """Load (once) and type the C ABI.  Raises loudly when the library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("MMSBM_LIB", path)  # measurement builds (tools/); default: in-tree build
    if not os.path.exists(path):
        raise ImportError("libmmsbm.so not built at %s: run "
                          "`python -m trigenicinteractionpredictor_amd.build`" % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def build_id() -> str:
    """The loaded library's build id (include/mmsbm.h, mmsbm_build_id)."""
    return load().mmsbm_build_id().decode()


def check(rc: int) -> None:
    if rc != MMSBM_OK:
        msg = load().mmsbm_last_error().decode(errors="replace")
        if rc == MMSBM_ERR_ZERO_DEGREE:
            raise ZeroDivisionError("float division by zero")
        raise MMSBMError(rc, msg)
