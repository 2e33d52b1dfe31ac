"""The fused K-layer forward as one device call (torch is only the memory/stream plumbing).

`dladmm_forward` packs the per-layer parameters into the tables the C ABI expects, allocates the
outputs and the workspace with torch on the current device, and enqueues
`dladmm_fwd_f32` (include/dladmm.h) on torch's current HIP stream.  There is no CPU fallback:
CPU tensors or a missing library raise.
"""
from __future__ import annotations

import contextlib
import contextvars
import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from . import _lib


@dataclass
class ForwardResult:
    Z: torch.Tensor          # [K | 1, n, B]
    E: torch.Tensor          # [K | 1, m, B]
    L: torch.Tensor          # [K | 1, m, B]
    T: Optional[torch.Tensor]  # [K+1 | 1, m, B] or None
    loss_sums: Optional[torch.Tensor]  # [K, 2] fp64: (sum|Z_k|, fit_k)
    col_loss: Optional[torch.Tensor] = None  # [K, 2, B] fp32 per-column terms (want_col_loss)
    P: Optional[torch.Tensor] = None  # [K, m, B] A Z_k per layer (want_P: training forwards)
    path: int = 0  # dladmm_fwd_path: the kernel path that ran (1 fused, 2 per-layer, 3 bf16
                   # tiles, 4 fused split-f16, 5 fused row-split, 6 its four-workgroup
                   # form; 0 = nothing launched)
    flags: int = 0  # the plan options (dladmm_flags) the forward ran with; its backward keeps them


_PLAN_FLAGS = contextvars.ContextVar("dladmm_plan_flags", default=0)
_FLAG_NAMES = {"per_layer": _lib.F_PER_LAYER, "bf16_wide": _lib.F_BF16_WIDE,
               "bwd_per_layer": _lib.F_BWD_PER_LAYER, "bwd_unfused": _lib.F_BWD_UNFUSED,
               "bwd_no_zmask": _lib.F_BWD_NO_ZMASK, "wgrad_f32": _lib.F_WGRAD_F32,
               "no_rowsplit": _lib.F_NO_ROWSPLIT, "no_xsplit": _lib.F_NO_XSPLIT}


@contextlib.contextmanager
def plan_flags(**opts):
    """Plan options (include/dladmm.h enum dladmm_flags) for every forward / backward call made
    inside the block, e.g. `with plan_flags(per_layer=True): net(X)` runs the per-layer kernels
    where the fused kernel would fit.  They select kernels, never arithmetic; the C ABI receives
    them in dladmm_fwd_desc.flags (the library reads no environment).  Nested blocks add to the
    enclosing block's flags; a False value clears that flag.  A backward keeps the options its
    forward ran with (ForwardResult.flags; autograd runs backwards on worker threads, outside
    the block) and adds those of a block around the backward call itself."""
    flags = _PLAN_FLAGS.get()
    for k, v in opts.items():
        if k not in _FLAG_NAMES:
            raise ValueError(f"dladmm: unknown plan flag {k!r} (one of {sorted(_FLAG_NAMES)})")
        flags = (flags | _FLAG_NAMES[k]) if v else (flags & ~_FLAG_NAMES[k])
    tok = _PLAN_FLAGS.set(flags)
    try:
        yield flags
    finally:
        _PLAN_FLAGS.reset(tok)


def _f32_dev(t: torch.Tensor, name: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"dladmm: {name} must be a tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"dladmm: {name} is on {t.device}; the fused forward runs on a HIP "
                           "device only (no CPU fallback)")
    if t.dtype != torch.float32:
        raise TypeError(f"dladmm: {name} must be float32, got {t.dtype}")
    if t.dim() != 2 or (t.stride(1) != 1 and t.numel() > 0):  # empty: strides are moot
        raise ValueError(f"dladmm: {name} must be a 2-D row-major matrix (batch contiguous)")
    return t


def _fill_fwd_desc(d, variant, X, A, W, Z0, E0, L0, scalar_params, row_params, beta1_elem,
                   beta2_elem, keep_all, loss_kind, out, flags=None):
    """Validate the forward's tensors and fill the C descriptor `d` (a FwdDesc, possibly embedded
    in a BwdDesc).  Returns the ctypes arrays that must outlive the call."""
    X = _f32_dev(X, "X")
    A = _f32_dev(A, "A")
    Z0, E0, L0 = _f32_dev(Z0, "Z0"), _f32_dev(E0, "E0"), _f32_dev(L0, "L0")
    m, B = X.shape
    n = A.shape[1]
    K = len(W)
    if A.shape[0] != m:
        raise RuntimeError(f"dladmm: A is {tuple(A.shape)} but X has {m} rows")
    if tuple(Z0.shape) != (n, B) or tuple(E0.shape) != (m, B) or tuple(L0.shape) != (m, B):
        raise RuntimeError(
            "dladmm: Z0/E0/L0 shapes do not broadcast with X: "
            f"Z0 {tuple(Z0.shape)}, E0 {tuple(E0.shape)}, L0 {tuple(L0.shape)}, X {tuple(X.shape)}")
    if not 1 <= K <= _lib.MAX_LAYERS:
        raise ValueError(f"dladmm: layers must be in [1, {_lib.MAX_LAYERS}], got {K}")
    Ws = [_f32_dev(w if w.dim() == 2 and w.stride(1) == 1 else w.contiguous(), f"W[{k}]")
          for k, w in enumerate(W)]
    ldw = Ws[0].stride(0)
    for k, w in enumerate(Ws):
        if tuple(w.shape) != (n, m) or w.stride(0) != ldw:
            raise RuntimeError(f"dladmm: fc[{k}].weight must be ({n}, {m}) with a common stride")
    dev = X.device
    d.abi_version = _lib.ABI_VERSION
    d.flags = _PLAN_FLAGS.get() if flags is None else int(flags)
    d.variant, d.m, d.n, d.batch, d.layers = variant, m, n, B, K
    d.keep_all, d.loss_kind = int(bool(keep_all)), int(loss_kind)
    d.X, d.ld_x = X.data_ptr(), X.stride(0)
    d.A, d.ld_a = A.data_ptr(), A.stride(0)
    d.Z0, d.ld_z0 = Z0.data_ptr(), Z0.stride(0)
    d.E0, d.ld_e0 = E0.data_ptr(), E0.stride(0)
    d.L0, d.ld_l0 = L0.data_ptr(), L0.stride(0)
    warr = _lib.ptr_array([w.data_ptr() for w in Ws])
    d.W, d.ld_w = ctypes.cast(warr, ctypes.POINTER(ctypes.c_void_p)), ldw
    keep = [warr, Ws]
    if scalar_params is not None:
        sp = scalar_params
        if sp.device != dev or sp.dtype != torch.float32 or tuple(sp.shape) != (K, _lib.NSCALAR) \
                or not sp.is_contiguous():
            raise ValueError("dladmm: scalar_params must be a contiguous (K, 8) fp32 device tensor")
        d.scalar_params = sp.data_ptr()
    if row_params is not None:
        rp = row_params
        if rp.device != dev or rp.dtype != torch.float32 or rp.dim() != 3 or \
                rp.shape[0] != K or rp.shape[1] != _lib.NSCALAR or not rp.is_contiguous():
            raise ValueError("dladmm: row_params must be a contiguous (K, 8, R) fp32 device tensor")
        d.row_params, d.row_stride = rp.data_ptr(), rp.shape[2]
    if len(beta1_elem):
        b1 = [_f32_dev(b, f"beta1[{k}]") for k, b in enumerate(beta1_elem)]
        b2 = [_f32_dev(b, f"beta2[{k}]") for k, b in enumerate(beta2_elem)]
        ldb = b1[0].stride(0)
        for b in b1 + b2:
            if tuple(b.shape) != (m, B) or b.stride(0) != ldb:
                raise RuntimeError(
                    f"dladmm: per-sample beta of shape {tuple(b.shape)} does not broadcast with "
                    f"X {tuple(X.shape)} (main_lena.py:35-36 betas are (m, batch_size))")
        a1 = _lib.ptr_array([b.data_ptr() for b in b1])
        a2 = _lib.ptr_array([b.data_ptr() for b in b2])
        keep += [a1, a2]
        d.beta1_elem = ctypes.cast(a1, ctypes.POINTER(ctypes.c_void_p))
        d.beta2_elem = ctypes.cast(a2, ctypes.POINTER(ctypes.c_void_p))
        d.ld_beta = ldb
    d.Z, d.E, d.L = out.Z.data_ptr(), out.E.data_ptr(), out.L.data_ptr()
    d.T = out.T.data_ptr() if out.T is not None else None
    d.ld_out = B
    d.loss_sums = out.loss_sums.data_ptr() if out.loss_sums is not None else None
    d.P = out.P.data_ptr() if out.P is not None else None
    return keep


# GEMM precision modes (include/dladmm.h, dladmm_precision): "f32" fp32 MFMA (exact fp32 fma
# chain); "f32_split" the same fp32 GEMMs on the f16 matrix cores (operands split exactly into
# power-of-two-scaled hi + lo halves, three products, fp32 accumulation: fp32-GEMM error);
# "bf16" bf16 operands (BASELINE config 5).
_PRECISIONS = {"f32": _lib.PREC_F32, "f32_split": _lib.PREC_F32_SPLIT, "bf16": _lib.PREC_BF16}


def dladmm_forward(variant: int, X: torch.Tensor, A: torch.Tensor, W: Sequence[torch.Tensor],
                   Z0: torch.Tensor, E0: torch.Tensor, L0: torch.Tensor, *,
                   scalar_params: Optional[torch.Tensor] = None,
                   row_params: Optional[torch.Tensor] = None,
                   beta1_elem: Sequence[torch.Tensor] = (),
                   beta2_elem: Sequence[torch.Tensor] = (),
                   keep_all: bool = True, want_T: bool = True, loss_kind: int = 0,
                   out: Optional[ForwardResult] = None,
                   kernel_events: Optional[tuple] = None,
                   want_col_loss: bool = False, precision: str = "f32",
                   want_P: bool = False, flags: Optional[int] = None) -> ForwardResult:
    """Run the whole K-layer forward of `variant` (dladmm_variant) on X's device.

    X: (m, B); A: (m, n); W: K tensors (n, m) (fc[k].weight; V5 passes the shared one K times);
    Z0: (n, B); E0, L0: (m, B).  scalar_params: (K, 8) device fp32 (V1, V4-V6);
    row_params: (K, 8, max(m, n)) (V2, V3); beta{1,2}_elem: K tensors (m, B) (V1).
    Returns views-ready stacked outputs and, if loss_kind, the per-layer (sum|Z|, fit) sums.
    want_P (training): also keep P_k = A Z_k of every layer (result.P) when the call runs on the
    fused fp32 kernel, so the backward reads the product instead of recomputing it; on every
    other path result.P stays None and the backward recomputes it.
    flags: plan options (include/dladmm.h dladmm_flags); None = those of the enclosing
    plan_flags block.
    """
    L = _lib.lib()
    _f32_dev(X, "X")
    _f32_dev(A, "A")
    m, B = X.shape
    n = A.shape[1]
    K = len(W)
    dev = X.device
    Kout = K if keep_all else 1
    if out is None:
        Zo = torch.empty((Kout, n, B), device=dev, dtype=torch.float32)
        Eo = torch.empty((Kout, m, B), device=dev, dtype=torch.float32)
        Lo = torch.empty((Kout, m, B), device=dev, dtype=torch.float32)
        To = (torch.empty((Kout + 1 if keep_all else 1, m, B), device=dev, dtype=torch.float32)
              if want_T else None)
        ls = torch.empty((K, 2), device=dev, dtype=torch.float64) if loss_kind else None
        out = ForwardResult(Zo, Eo, Lo, To, ls)
    out.flags = _PLAN_FLAGS.get() if flags is None else int(flags)

    if B == 0:
        # an empty batch: the reference's ops return empty (rows, 0) tensors and zero sums; no
        # kernel runs (shapes are still checked)
        _fill_fwd_desc(_lib.FwdDesc(), variant, X, A, W, Z0, E0, L0, scalar_params, row_params,
                       beta1_elem, beta2_elem, keep_all, loss_kind, out, out.flags)
        if out.loss_sums is not None:
            out.loss_sums.zero_()
        if want_col_loss:
            out.col_loss = torch.zeros((K, 2, 0), device=dev, dtype=torch.float32)
        if want_P and keep_all:
            out.P = torch.empty((K, m, 0), device=dev, dtype=torch.float32)
        return out
    d = _lib.FwdDesc()
    keep = _fill_fwd_desc(d, variant, X, A, W, Z0, E0, L0, scalar_params, row_params, beta1_elem,
                          beta2_elem, keep_all, loss_kind, out, out.flags)
    if precision not in _PRECISIONS:
        raise ValueError(f"dladmm: precision must be one of {sorted(_PRECISIONS)}, "
                         f"got {precision!r}")
    d.precision = _PRECISIONS[precision]
    # (path 5, the small-batch row-split kernel, saves no product: with P set the plan is path 1)
    if want_P and keep_all and out.P is None and L.dladmm_fwd_path(ctypes.byref(d)) in (1, 4, 5, 6):
        out.P = torch.empty((K, m, B), device=dev, dtype=torch.float32)
        d.P = out.P.data_ptr()
    if want_col_loss:
        if not loss_kind:
            raise ValueError("dladmm: per-column objectives need loss_kind")
        if out.col_loss is None:
            out.col_loss = torch.empty((K, 2, B), device=dev, dtype=torch.float32)
        d.col_loss = out.col_loss.data_ptr()
    if kernel_events is not None:  # (torch.cuda.Event, torch.cuda.Event) around the fused kernel
        d.ev_kernel_start = kernel_events[0].cuda_event
        d.ev_kernel_stop = kernel_events[1].cuda_event

    wsb = L.dladmm_fwd_workspace_bytes(ctypes.byref(d))
    if wsb == 0:
        path = L.dladmm_fwd_path(ctypes.byref(d))
        _lib.check(path if path < 0 else -7)
    out.path = L.dladmm_fwd_path(ctypes.byref(d))
    ws = _workspace(dev, wsb)
    d.workspace, d.workspace_bytes = ws.data_ptr(), wsb
    stream = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(L.dladmm_fwd_f32(ctypes.byref(d), ctypes.c_void_p(stream)))
    del keep
    return out


@dataclass
class BackwardResult:
    gW: torch.Tensor                  # [K, n, m] (V5 tied: [1, n, m])
    g_scalar: Optional[torch.Tensor]  # [K, 8] fp64 (V4-V6)
    g_row: Optional[torch.Tensor]     # [K, 8, R] fp64 (V2, V3)
    g_beta1: List[torch.Tensor]       # V1: K tensors (m, B)
    g_beta2: List[torch.Tensor]
    path: int = 0                     # dladmm_bwd_path: 1 = one reverse-sweep kernel (2: its
                                      # small-batch row-split form, 3: that over four
                                      # workgroups per 16 columns), 0 = per layer


def dladmm_backward(variant: int, X: torch.Tensor, A: torch.Tensor, W: Sequence[torch.Tensor],
                    Z0: torch.Tensor, E0: torch.Tensor, L0: torch.Tensor, saved: ForwardResult,
                    gZ: Optional[Sequence] = None, gE: Optional[Sequence] = None,
                    gL: Optional[Sequence] = None, gT: Optional[Sequence] = None, *,
                    loss_kind: int = 0, loss_coef: Optional[torch.Tensor] = None,
                    scalar_params: Optional[torch.Tensor] = None,
                    row_params: Optional[torch.Tensor] = None,
                    beta1_elem: Sequence[torch.Tensor] = (),
                    beta2_elem: Sequence[torch.Tensor] = (),
                    tied: bool = False, flags: Optional[int] = None) -> BackwardResult:
    """Gradients of sum_k <gZ_k,Z_k> + <gE_k,E_k> + <gL_k,L_k> + sum_j <gT_j,T_j> (+ the fused
    training objective sum_k cz_k sum|Z_k| + cf_k fit_k when loss_kind, loss_coef = device
    (K, 2) fp32 (cz_k, cf_k)) w.r.t. the parameters of the forward that produced `saved` (a
    keep_all ForwardResult with T), via `dladmm_bwd_f32` (include/dladmm.h).  Cotangents are
    per-layer sequences of (rows, B) tensors (None entries / None = zero).  This is the backward
    of the reference's `total_loss.backward()` through DLADMMNet.forward
    (main_syn_l1l1_scalar.py:298).  flags: plan options; None = the forward's (saved.flags)
    plus those of an enclosing plan_flags block."""
    L = _lib.lib()
    if saved.T is None or saved.Z.shape[0] != len(W):
        raise ValueError("dladmm: backward needs the keep_all forward outputs including T")
    m, B = X.shape
    n = A.shape[1]
    K = len(W)
    dev = X.device
    if B == 0:  # an empty batch contributes nothing to any gradient
        gs = torch.zeros((K, _lib.NSCALAR), device=dev, dtype=torch.float64) \
            if variant >= _lib.V4_SCALAR else None
        gr = torch.zeros((K, _lib.NSCALAR, row_params.shape[2]), device=dev,
                         dtype=torch.float64) if variant in (_lib.V2_LTHETA, _lib.V3_FULL) else None
        gb = [torch.zeros((m, 0), device=dev) for _ in range(K)] if variant == _lib.V1_LENA \
            else []
        return BackwardResult(torch.zeros((1 if tied else K, n, m), device=dev), gs, gr, gb,
                              [t.clone() for t in gb])
    d = _lib.BwdDesc()
    if flags is None:
        flags = int(getattr(saved, "flags", 0)) | _PLAN_FLAGS.get()
    keep = _fill_fwd_desc(d.fwd, variant, X, A, W, Z0, E0, L0, scalar_params, row_params,
                          beta1_elem, beta2_elem, True, 0, saved, flags)
    # a split-f16 training forward (path 4) also runs the weight-gradient GEMM on the f16
    # matrix cores (csrc/dladmm_wgrad_x3.hip); every other backward kernel is the fp32 one
    d.fwd.precision = _PRECISIONS["f32_split"] if saved.path == 4 else _PRECISIONS["f32"]
    counts = {"gZ": (K, n), "gE": (K, m), "gL": (K, m), "gT": (K + 1, m)}
    for nm, seq in (("gZ", gZ), ("gE", gE), ("gL", gL), ("gT", gT)):
        if seq is None or all(g is None for g in seq):
            continue
        cnt, rows = counts[nm]
        if len(seq) != cnt:
            raise ValueError(f"dladmm: {nm} must have {cnt} entries")
        ptrs = []
        for g in seq:
            if g is None:
                ptrs.append(None)
                continue
            if tuple(g.shape) != (rows, B) or g.dtype != torch.float32 or g.device != dev:
                raise ValueError(f"dladmm: {nm} entries must be fp32 ({rows}, {B}) device tensors")
            g = g.contiguous()
            keep.append(g)
            ptrs.append(g.data_ptr())
        arr = _lib.ptr_array(ptrs)
        keep.append(arr)
        setattr(d, nm, ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)))
    d.ld_g = B
    if loss_kind:
        if loss_coef is None or tuple(loss_coef.shape) != (K, 2) or loss_coef.dtype != \
                torch.float32 or loss_coef.device != dev or not loss_coef.is_contiguous():
            raise ValueError("dladmm: loss_coef must be a contiguous fp32 (K, 2) device tensor")
        d.loss_kind, d.loss_coef = int(loss_kind), loss_coef.data_ptr()
    gWo = torch.empty((1 if tied else K, n, m), device=dev, dtype=torch.float32)
    d.gW, d.ld_gw = gWo.data_ptr(), m
    d.gw_sum = int(bool(tied))
    g_scalar = g_row = None
    g1, g2 = [], []
    if variant >= _lib.V4_SCALAR:
        g_scalar = torch.zeros((K, _lib.NSCALAR), device=dev, dtype=torch.float64)
        d.g_scalar = g_scalar.data_ptr()
    elif variant in (_lib.V2_LTHETA, _lib.V3_FULL):
        g_row = torch.zeros((K, _lib.NSCALAR, d.fwd.row_stride), device=dev, dtype=torch.float64)
        d.g_row = g_row.data_ptr()
    else:
        g1 = [torch.empty((m, B), device=dev, dtype=torch.float32) for _ in range(K)]
        g2 = [torch.empty((m, B), device=dev, dtype=torch.float32) for _ in range(K)]
        if d.fwd.ld_beta != B:
            raise ValueError("dladmm: V1 backward needs contiguous (m, B) betas")
        a1 = _lib.ptr_array([t.data_ptr() for t in g1])
        a2 = _lib.ptr_array([t.data_ptr() for t in g2])
        keep += [a1, a2]
        d.g_beta1_elem = ctypes.cast(a1, ctypes.POINTER(ctypes.c_void_p))
        d.g_beta2_elem = ctypes.cast(a2, ctypes.POINTER(ctypes.c_void_p))
    wsb = L.dladmm_bwd_workspace_bytes(ctypes.byref(d))
    if wsb == 0:
        raise ValueError("dladmm: invalid backward descriptor")
    path = L.dladmm_bwd_path(ctypes.byref(d))
    ws = _workspace(dev, wsb)
    d.workspace, d.workspace_bytes = ws.data_ptr(), wsb
    stream = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(L.dladmm_bwd_f32(ctypes.byref(d), ctypes.c_void_p(stream)))
    del keep
    return BackwardResult(gWo, g_scalar, g_row, g1, g2, path)


def dladmm_scale_(x: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """x *= s in place (s: a one-element fp32 device tensor) through dladmm_scale_f32, which skips
    the pass on the device when s == 1 -- no host synchronisation."""
    if x.dtype != torch.float32 or not x.is_contiguous() or s.dtype != torch.float32 or \
            s.numel() != 1 or s.device != x.device or x.device.type != "cuda":
        raise ValueError("dladmm: scale needs a contiguous fp32 tensor and an fp32 device scalar")
    s = s.contiguous()
    stream = torch.cuda.current_stream(x.device).cuda_stream
    _lib.check(_lib.lib().dladmm_scale_f32(ctypes.c_void_p(x.data_ptr()), x.numel(),
                                           ctypes.c_void_p(s.data_ptr()), ctypes.c_void_p(stream)))
    return x


def dladmm_lena(X: torch.Tensor, A: torch.Tensor, E: torch.Tensor, L: torch.Tensor, alpha: float,
                denom: float, coef: Optional[torch.Tensor] = None, sums: bool = True,
                lx_sign: float = 1.0):
    """The fused main_lena.py objective terms over a forward's saved E_k, L_k ((K, m, B) each;
    main_lena.py:221-228 with dual_gap :145-147) through `dladmm_lena_f32` (include/dladmm.h,
    csrc/dladmm_lena.hip).  coef None (mode 0): returns the fp64 (K, 4) sums
    [sum|E_k|, sum dual_gap(A^T L_k, alpha), sum dual_gap(L_k, 1), sum L_k X].  coef = device
    fp32 (K,) (mode 1): returns the cotangents (gE, gL), each (K, m, B), of
    sum_k coef[k] * (mean|E_k| + mean dual_gap(A^T L_k, alpha) + mean dual_gap(L_k, 1)
    + lx_sign mean(L_k X)), the means over m*denom (n*denom for A^T L_k) elements; with coef and
    sums (mode 2, one pass) returns (sums, gE, gL).  lx_sign: +1 main_lena.py:226, -1
    main_syn_l1l1-dgap_ltheta.py:205 (the sums are unsigned either way)."""
    Lb = _lib.lib()
    if lx_sign not in (1.0, -1.0):
        raise ValueError(f"dladmm: lx_sign must be +1 or -1 (got {lx_sign})")
    K, m, B = L.shape
    n = A.shape[1]
    dev = X.device
    for t in (E, L):
        if tuple(t.shape) != (K, m, B) or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("dladmm: E and L must be contiguous fp32 (K, m, B) tensors")
    if tuple(X.shape) != (m, B) or tuple(A.shape) != (m, n) or X.dtype != torch.float32 or \
            A.dtype != torch.float32:
        raise ValueError(f"dladmm: X must be fp32 ({m}, {B}) and A fp32 ({m}, n); got "
                         f"{tuple(X.shape)} {X.dtype}, {tuple(A.shape)} {A.dtype}")
    if dev.type != "cuda" or any(t.device != dev for t in (A, E, L)):
        raise ValueError("dladmm: X, A, E and L must be on one GPU")
    if K == 0 or B == 0:   # nothing to reduce: zero sums, empty cotangents, no launch
        sm = torch.zeros((K, 4), device=dev, dtype=torch.float64)
        gE, gL = torch.zeros_like(E), torch.zeros_like(L)
        if coef is None:
            return sm
        return (sm, gE, gL) if sums else (gE, gL)
    X = X.contiguous()
    A = A.contiguous()
    d = _lib.LenaDesc()
    d.abi_version = _lib.ABI_VERSION
    d.m, d.n, d.batch, d.layers = m, n, B, K
    d.alpha = float(alpha)
    d.lx_negate = 1 if lx_sign < 0 else 0
    d.inv_mb, d.inv_nb = 1.0 / (m * float(denom)), 1.0 / (n * float(denom))
    d.X, d.ld_x = X.data_ptr(), X.stride(0)
    d.A, d.ld_a = A.data_ptr(), A.stride(0)
    d.E, d.L, d.layer_stride, d.ld = E.data_ptr(), L.data_ptr(), m * B, B
    sm = gE = gL = None
    if coef is None or sums:
        sm = torch.empty((K, 4), device=dev, dtype=torch.float64)
        d.sums = sm.data_ptr()
    if coef is not None:
        if tuple(coef.shape) != (K,) or coef.dtype != torch.float32 or coef.device != dev:
            raise ValueError("dladmm: coef must be an fp32 (K,) device tensor")
        coef = coef.contiguous()
        gE = torch.empty((K, m, B), device=dev, dtype=torch.float32)
        gL = torch.empty((K, m, B), device=dev, dtype=torch.float32)
        d.gE, d.gL, d.g_layer_stride, d.ld_g = gE.data_ptr(), gL.data_ptr(), m * B, B
        d.coef = coef.data_ptr()
    d.mode = 0 if coef is None else (2 if sums else 1)
    out = sm if coef is None else ((sm, gE, gL) if sums else (gE, gL))
    wsb = Lb.dladmm_lena_workspace_bytes(ctypes.byref(d))
    if wsb == 0:
        raise ValueError(f"dladmm: the fused main_lena objective supports m <= 256, n <= 512 "
                         f"(got m={m}, n={n}, K={K}, B={B})")
    ws = _workspace(dev, wsb)
    d.workspace, d.workspace_bytes = ws.data_ptr(), wsb
    stream = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(Lb.dladmm_lena_f32(ctypes.byref(d), ctypes.c_void_p(stream)))
    return out


_WS: "OrderedDict" = None
_WS_PER_DEVICE = 4   # streams whose workspace stays cached per device (least recently used out)


def _workspace(dev: torch.device, nbytes: int) -> torch.Tensor:
    """Cached workspace per (device, stream), grown on demand (torch's allocator keeps it 256-B
    aligned).  Reuse is safe because it is stream-ordered: a buffer is only ever used by calls
    enqueued on the stream it was allocated on, so two streams of one device (say overlapping
    eval and training) never share scratch memory, and a buffer dropped when it grows -- or when
    its stream falls out of the cache -- goes back to the caching allocator under the one stream
    that used it.  At most _WS_PER_DEVICE streams per device keep a buffer (least recently used
    evicted), so code that makes a new stream per pass does not grow memory without bound."""
    global _WS
    from collections import OrderedDict
    if _WS is None:
        _WS = OrderedDict()
    stream = torch.cuda.current_stream(dev)
    key = (dev.type, dev.index, stream.cuda_stream)
    buf = _WS.pop(key, None)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1), device=dev, dtype=torch.uint8)
    _WS[key] = buf   # most recently used last
    same = [k for k in _WS if k[:2] == key[:2]]
    for k in same[:-_WS_PER_DEVICE]:
        del _WS[k]
    return buf
