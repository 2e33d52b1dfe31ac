"""ctypes binding of the C ABI in include/dladmm.h (libdladmm_hip.so, built in-tree).

No torch types cross this boundary: the descriptor carries raw device pointers, sizes and leading
dimensions; the stream is a hipStream_t passed as an integer.  The library is loaded lazily and
loading failures raise -- there is no fallback path.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DLADMM_LIB") or os.path.join(HERE, "lib", "libdladmm_hip.so")

ABI_VERSION = 6
PREC_F32, PREC_BF16, PREC_F32_SPLIT = 0, 1, 2
MAX_LAYERS = 65536
NSCALAR = 8

# enum dladmm_flags (dladmm_fwd_desc.flags): plan options, never arithmetic
F_PER_LAYER, F_BF16_WIDE, F_BWD_PER_LAYER, F_BWD_UNFUSED, F_BWD_NO_ZMASK, F_WGRAD_F32 = \
    1, 2, 4, 8, 16, 32
F_NO_ROWSPLIT = 64
F_NO_XSPLIT = 128
# enum dladmm_variant
V1_LENA, V2_LTHETA, V3_FULL, V4_SCALAR, V5_TIED, V6_LASSO = 1, 2, 3, 4, 5, 6
# enum dladmm_loss_kind
LOSS_NONE, LOSS_L1L1, LOSS_LASSO = 0, 1, 2
# enum dladmm_param_slot
P_BETA1, P_BETA2, P_BETA3, P_SS2, P_SS2B, P_THETA_E, P_THETA_Z, P_S1 = range(8)

# every symbol include/dladmm.h declares (checked by tests/test_capi.py)
EXPORTED = ("dladmm_abi_version", "dladmm_fwd_workspace_bytes", "dladmm_fwd_path",
            "dladmm_fwd_f32", "dladmm_bwd_workspace_bytes", "dladmm_bwd_path", "dladmm_bwd_f32",
            "dladmm_safeguard_f32", "dladmm_colobj_f32", "dladmm_lena_workspace_bytes",
            "dladmm_lena_f32", "dladmm_scale_f32", "dladmm_error_string")
# enum dladmm_mu_updater
MU_NONE, MU_EMA, MU_GS, MU_RT = 0, 1, 2, 3

_fp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64


class FwdDesc(ctypes.Structure):
    """Mirror of `struct dladmm_fwd_desc` (include/dladmm.h)."""
    _fields_ = [
        ("abi_version", _i32), ("variant", _i32), ("m", _i32), ("n", _i32),
        ("batch", _i32), ("layers", _i32), ("keep_all", _i32), ("loss_kind", _i32),
        ("X", _fp), ("ld_x", _i64),
        ("A", _fp), ("ld_a", _i64),
        ("Z0", _fp), ("ld_z0", _i64),
        ("E0", _fp), ("ld_e0", _i64),
        ("L0", _fp), ("ld_l0", _i64),
        ("W", ctypes.POINTER(_fp)), ("ld_w", _i64),
        ("scalar_params", _fp),
        ("row_params", _fp), ("row_stride", _i64),
        ("beta1_elem", ctypes.POINTER(_fp)),
        ("beta2_elem", ctypes.POINTER(_fp)),
        ("ld_beta", _i64),
        ("Z", _fp), ("E", _fp), ("L", _fp), ("T", _fp),
        ("ld_out", _i64),
        ("loss_sums", _fp),
        ("workspace", _fp), ("workspace_bytes", ctypes.c_size_t),
        ("ev_kernel_start", _fp), ("ev_kernel_stop", _fp),
        ("col_loss", _fp),
        ("precision", _i32), ("flags", _i32),
        ("P", _fp),
    ]


class BwdDesc(ctypes.Structure):
    """Mirror of `struct dladmm_bwd_desc` (include/dladmm.h)."""
    _fields_ = [
        ("fwd", FwdDesc),
        ("gZ", ctypes.POINTER(_fp)), ("gE", ctypes.POINTER(_fp)), ("gL", ctypes.POINTER(_fp)),
        ("gT", ctypes.POINTER(_fp)), ("ld_g", _i64),
        ("loss_kind", _i32), ("gw_sum", _i32), ("loss_coef", _fp),
        ("gW", _fp), ("ld_gw", _i64),
        ("g_scalar", _fp), ("g_row", _fp),
        ("g_beta1_elem", ctypes.POINTER(_fp)), ("g_beta2_elem", ctypes.POINTER(_fp)),
        ("workspace", _fp), ("workspace_bytes", ctypes.c_size_t),
    ]


class SafeguardDesc(ctypes.Structure):
    """Mirror of `struct dladmm_safeguard_desc` (include/dladmm.h)."""
    _fields_ = [
        ("abi_version", _i32), ("m", _i32), ("n", _i32), ("batch", _i32), ("ld", _i64),
        ("Zl", _fp), ("El", _fp), ("Ll", _fp), ("Tl", _fp),
        ("Zk", _fp), ("Ek", _fp), ("Lk", _fp), ("Tk", _fp),
        ("Es", _fp), ("Ts", _fp), ("Ep", _fp),
        ("Zo", _fp), ("Eo", _fp), ("Lo", _fp), ("To", _fp),
        ("mu", _fp), ("norm_out", _fp), ("count", _fp),
        ("beta", ctypes.c_float), ("c", ctypes.c_float), ("delta", ctypes.c_double),
        ("updater", _i32), ("mu_param", ctypes.c_float),
    ]


class ColObjDesc(ctypes.Structure):
    """Mirror of `struct dladmm_colobj_desc` (include/dladmm.h)."""
    _fields_ = [
        ("abi_version", _i32), ("m", _i32), ("n", _i32), ("batch", _i32), ("layers", _i32),
        ("fit_kind", _i32),
        ("Z", _fp), ("z_layer_stride", _i64), ("ld_z", _i64),
        ("E", _fp), ("e_layer_stride", _i64), ("ld_e", _i64),
        ("T", _fp), ("t_layer_stride", _i64), ("ld_t", _i64),
        ("Zref", _fp), ("ld_zref", _i64),
        ("Eref", _fp), ("ld_eref", _i64),
        ("reg", _fp), ("fit", _fp), ("dz", _fp), ("de", _fp),
    ]


class LenaDesc(ctypes.Structure):
    """Mirror of `struct dladmm_lena_desc` (include/dladmm.h)."""
    _fields_ = [
        ("abi_version", _i32), ("m", _i32), ("n", _i32), ("batch", _i32), ("layers", _i32),
        ("mode", _i32), ("alpha", ctypes.c_float), ("inv_mb", ctypes.c_float),
        ("inv_nb", ctypes.c_float), ("lx_negate", _i32),
        ("X", _fp), ("ld_x", _i64), ("A", _fp), ("ld_a", _i64),
        ("E", _fp), ("L", _fp), ("layer_stride", _i64), ("ld", _i64),
        ("sums", _fp),
        ("gE", _fp), ("gL", _fp), ("g_layer_stride", _i64), ("ld_g", _i64),
        ("coef", _fp),
        ("workspace", _fp), ("workspace_bytes", ctypes.c_size_t),
    ]


_LIB = None


def lib():
    """Load libdladmm_hip.so (after torch, so it binds torch's HIP runtime by SONAME)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"dladmm: HIP library not built ({LIB_PATH} missing); run "
            "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C d-ladmm_amd`")
    import torch  # noqa: F401  -- makes torch's libamdhip64 the process-wide HIP runtime
    L = ctypes.CDLL(LIB_PATH)
    L.dladmm_abi_version.restype = ctypes.c_int
    L.dladmm_abi_version.argtypes = []
    L.dladmm_fwd_workspace_bytes.restype = ctypes.c_size_t
    L.dladmm_fwd_workspace_bytes.argtypes = [ctypes.POINTER(FwdDesc)]
    L.dladmm_fwd_path.restype = ctypes.c_int
    L.dladmm_fwd_path.argtypes = [ctypes.POINTER(FwdDesc)]
    L.dladmm_fwd_f32.restype = ctypes.c_int
    L.dladmm_fwd_f32.argtypes = [ctypes.POINTER(FwdDesc), ctypes.c_void_p]
    L.dladmm_bwd_workspace_bytes.restype = ctypes.c_size_t
    L.dladmm_bwd_workspace_bytes.argtypes = [ctypes.POINTER(BwdDesc)]
    L.dladmm_bwd_path.restype = ctypes.c_int
    L.dladmm_bwd_path.argtypes = [ctypes.POINTER(BwdDesc)]
    L.dladmm_bwd_f32.restype = ctypes.c_int
    L.dladmm_bwd_f32.argtypes = [ctypes.POINTER(BwdDesc), ctypes.c_void_p]
    L.dladmm_safeguard_f32.restype = ctypes.c_int
    L.dladmm_safeguard_f32.argtypes = [ctypes.POINTER(SafeguardDesc), ctypes.c_void_p]
    L.dladmm_colobj_f32.restype = ctypes.c_int
    L.dladmm_colobj_f32.argtypes = [ctypes.POINTER(ColObjDesc), ctypes.c_void_p]
    L.dladmm_lena_workspace_bytes.restype = ctypes.c_size_t
    L.dladmm_lena_workspace_bytes.argtypes = [ctypes.POINTER(LenaDesc)]
    L.dladmm_lena_f32.restype = ctypes.c_int
    L.dladmm_lena_f32.argtypes = [ctypes.POINTER(LenaDesc), ctypes.c_void_p]
    L.dladmm_scale_f32.restype = ctypes.c_int
    L.dladmm_scale_f32.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    L.dladmm_error_string.restype = ctypes.c_char_p
    L.dladmm_error_string.argtypes = [ctypes.c_int]
    if L.dladmm_abi_version() != ABI_VERSION:
        raise RuntimeError("dladmm: library ABI version mismatch; rebuild")
    _LIB = L
    return L


def check(code: int):
    if code != 0:
        msg = lib().dladmm_error_string(code).decode()
        if code < 0:
            raise ValueError(f"{msg} (code {code})")
        raise RuntimeError(f"dladmm HIP error: {msg} (code {code})")


def ptr_array(ptrs):
    arr = (_fp * max(len(ptrs), 1))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr
