"""The C-ABI library (include/dladmm.h) loads, exports every declared symbol and validates
descriptors -- CPU only, no compute call is made."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_symbols_exported(dl):
    L = dl._lib.lib()
    hdr = open(os.path.join(ROOT, "include", "dladmm.h")).read()
    declared = set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(dladmm_\w+)\s*\(", hdr, re.M))
    assert declared == set(dl._lib.EXPORTED)
    for sym in declared:
        assert hasattr(L, sym), sym
    assert L.dladmm_abi_version() == dl._lib.ABI_VERSION


def _desc(dl, **kw):
    F = dl._lib.FwdDesc
    d = F()
    d.abi_version = dl._lib.ABI_VERSION
    d.variant = dl._lib.V4_SCALAR
    d.m, d.n, d.batch, d.layers = 256, 512, 1000, 15
    d.keep_all, d.loss_kind = 1, 1
    fake = 1 << 40  # never dereferenced: only validation / sizing is exercised here
    for f in ("X", "A", "Z0", "E0", "L0", "scalar_params", "Z", "E", "L", "T", "loss_sums"):
        setattr(d, f, fake)
    d.ld_x = d.ld_z0 = d.ld_e0 = d.ld_l0 = d.ld_out = 1000
    d.ld_a, d.ld_w = 512, 256
    w = dl._lib.ptr_array([fake + 4096 * k for k in range(15)])
    d.W = ctypes.cast(w, ctypes.POINTER(ctypes.c_void_p))
    for k, v in kw.items():
        setattr(d, k, v)
    return d, w


def test_workspace_and_path(dl):
    L = dl._lib.lib()
    d, _keep = _desc(dl)
    # B = 1,000 at 256 x 512: the four-workgroup row split (path 6; its 256-workgroup grid fits
    # one per CU -- the plan assumes 256 CUs where no device answers); no_xsplit: the
    # one-workgroup row split (path 5, up to three per CU)
    assert L.dladmm_fwd_path(ctypes.byref(d)) == 6
    d.flags = dl._lib.F_NO_XSPLIT
    assert L.dladmm_fwd_path(ctypes.byref(d)) == 5
    d.flags = dl._lib.F_NO_ROWSPLIT
    assert L.dladmm_fwd_path(ctypes.byref(d)) == 1
    d.flags = 0
    big, _k2 = _desc(dl, batch=65536, ld_x=65536, ld_z0=65536, ld_e0=65536, ld_l0=65536,
                     ld_out=65536)
    assert L.dladmm_fwd_path(ctypes.byref(big)) == 1
    ws = L.dladmm_fwd_workspace_bytes(ctypes.byref(d))
    # packed A + 15 packed W_k (256 x 512 fp32 each) + per-wave loss partials
    assert ws >= 16 * 256 * 512 * 4 + 2 * 15 * 16 * 4 * 4
    assert ws % 256 == 0
    # one weight shared by every layer (V5 tied / the KM iteration) is packed once
    w1 = dl._lib.ptr_array([1 << 40] * 15)
    d.W = ctypes.cast(w1, ctypes.POINTER(ctypes.c_void_p))
    assert L.dladmm_fwd_workspace_bytes(ctypes.byref(d)) == ws - 14 * 256 * 512 * 4


@pytest.mark.parametrize("field,value,code", [
    ("abi_version", 99, -1), ("variant", 9, -2), ("m", 0, -3), ("batch", 0, -3),
    ("layers", 0, -4), ("layers", 65537, -4), ("X", None, -5), ("ld_x", 10, -3),
    ("loss_kind", 7, -7),
])
def test_validation_codes(dl, field, value, code):
    L = dl._lib.lib()
    d, _keep = _desc(dl, **{field: value})
    assert L.dladmm_fwd_path(ctypes.byref(d)) == code
    assert L.dladmm_fwd_workspace_bytes(ctypes.byref(d)) == 0
    assert L.dladmm_fwd_f32(ctypes.byref(d), None) == code
    assert L.dladmm_error_string(code).decode().startswith("dladmm:")


def test_large_shapes_take_the_per_layer_path(dl):
    """m > 256 or n > 512 (BASELINE config 4: 512 x 2048) exceed the fused kernel's register
    budget and run as per-layer kernel pairs (path 2)."""
    L = dl._lib.lib()
    d, _keep = _desc(dl, m=512, n=2048, ld_a=2048, ld_w=512, batch=65536, ld_x=65536,
                     ld_z0=65536, ld_e0=65536, ld_l0=65536, ld_out=65536)
    assert L.dladmm_fwd_path(ctypes.byref(d)) == 2
    assert L.dladmm_fwd_workspace_bytes(ctypes.byref(d)) > 15 * 2048 * 512 * 4


def _bdesc(dl, **kw):
    d, keep = _desc(dl)
    b = dl._lib.BwdDesc()
    b.fwd = d
    fake = 1 << 40
    b.gW, b.ld_gw = fake, 256
    b.g_scalar = fake
    gz = dl._lib.ptr_array([fake] * 15)
    b.gZ, b.ld_g = ctypes.cast(gz, ctypes.POINTER(ctypes.c_void_p)), 1000
    for k, v in kw.items():
        setattr(b, k, v)
    return b, (keep, gz)


def test_backward_workspace_and_validation(dl):
    L = dl._lib.lib()
    b, _keep = _bdesc(dl)
    ws = L.dladmm_bwd_workspace_bytes(ctypes.byref(b))
    # adjoint buffers (5 x m + padded n, padded m rows of padded batch) + packed A, A^T, M, M^T
    assert ws >= (5 * 256 + 512 + 256) * 1008 * 4 + 4 * 256 * 512 * 4
    assert ws % 256 == 0
    for field, value, code in (("gW", None, -5), ("g_scalar", None, -5), ("ld_g", 10, -3),
                               ("ld_gw", 100, -3), ("loss_kind", 1, -5), ("loss_kind", 5, -7)):
        bb, _k2 = _bdesc(dl, **{field: value})
        assert L.dladmm_bwd_workspace_bytes(ctypes.byref(bb)) == 0
        assert L.dladmm_bwd_f32(ctypes.byref(bb), None) == code, field
    # the forward must have saved every layer and T
    bb, _k3 = _bdesc(dl)
    bb.fwd.keep_all = 0
    assert L.dladmm_bwd_f32(ctypes.byref(bb), None) == -7
    bb.fwd.keep_all = 1
    bb.fwd.T = None
    assert L.dladmm_bwd_f32(ctypes.byref(bb), None) == -7


def test_plan_flags_select_kernels(dl):
    """dladmm_fwd_desc.flags (enum dladmm_flags) is the whole plan-option input: per_layer moves
    a fused-shape forward to the per-layer pair; bwd_per_layer moves a saved-product backward
    off the reverse sweep; unknown bits change nothing."""
    L = dl._lib.lib()
    d, _keep = _desc(dl)
    assert L.dladmm_fwd_path(ctypes.byref(d)) == 6
    d.flags = dl._lib.F_NO_XSPLIT
    assert L.dladmm_fwd_path(ctypes.byref(d)) == 5
    d.flags = dl._lib.F_NO_ROWSPLIT
    assert L.dladmm_fwd_path(ctypes.byref(d)) == 1
    d.flags = dl._lib.F_PER_LAYER
    assert L.dladmm_fwd_path(ctypes.byref(d)) == 2
    d.flags = 1 << 20
    assert L.dladmm_fwd_path(ctypes.byref(d)) == 6
    d.precision = dl._lib.PREC_BF16
    for f in (0, dl._lib.F_BF16_WIDE):
        d.flags = f
        assert L.dladmm_fwd_path(ctypes.byref(d)) == 3
    b, _k = _bdesc(dl)
    b.fwd.P = 1 << 40   # a saved-product forward (B = 1,000: path 6, the four-workgroup sweep)
    assert L.dladmm_bwd_path(ctypes.byref(b)) == 3
    b.fwd.flags = dl._lib.F_NO_XSPLIT   # a path-5 forward: the one-workgroup row-split sweep
    assert L.dladmm_bwd_path(ctypes.byref(b)) == 2
    b.fwd.flags = dl._lib.F_NO_ROWSPLIT   # a path-1 forward: the 64-column sweep
    assert L.dladmm_bwd_path(ctypes.byref(b)) == 1
    b.fwd.precision = dl._lib.PREC_F32_SPLIT   # a split-f16 forward (path 4) likewise
    b.fwd.flags = 0
    assert L.dladmm_bwd_path(ctypes.byref(b)) == 1
    b.fwd.precision = dl._lib.PREC_F32
    b.fwd.flags = dl._lib.F_BWD_PER_LAYER
    assert L.dladmm_bwd_path(ctypes.byref(b)) == 0
    assert L.dladmm_bwd_workspace_bytes(ctypes.byref(b)) > 0


def test_library_reads_no_environment(dl):
    """The product library imports no getenv: plan choices come from the descriptor only (the
    cycle-stamp diagnostic build, -DX3_STAMP, is the one exception and is never shipped)."""
    import shutil
    import subprocess
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    if not os.path.exists(nm) and not shutil.which(nm):
        pytest.skip("no nm")
    out = subprocess.run([nm, "-D", "--undefined-only", dl._lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert "getenv" not in out


def test_plan_flags_context():
    import importlib
    ops = importlib.import_module("d-ladmm_amd.ops")
    lib = importlib.import_module("d-ladmm_amd._lib")
    assert ops._PLAN_FLAGS.get() == 0
    with ops.plan_flags(per_layer=True) as f1:
        assert f1 == lib.F_PER_LAYER
        with ops.plan_flags(bwd_unfused=True, per_layer=False) as f2:
            assert f2 == lib.F_BWD_UNFUSED
        assert ops._PLAN_FLAGS.get() == lib.F_PER_LAYER
    assert ops._PLAN_FLAGS.get() == 0
    with pytest.raises(ValueError):
        with ops.plan_flags(no_such_flag=True):
            pass
