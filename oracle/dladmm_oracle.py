"""CPU restatement of the reference D-LADMM forward -- TEST INFRASTRUCTURE ONLY.

This module is the parity oracle.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it, and only as the checker / the timed CPU baseline.  The product
path (d-ladmm_amd/) never imports it and has no CPU fallback.

It restates, op for op and in the reference's evaluation order, the `DLADMMNet.forward` bodies of
the reference scripts (numpy, fp32 by default, fp64 on request):

  V1  main_lena.py:57-98            (per-sample beta (m,B), fixed thresholds 0.025 / 0.06)
  V2  main_syn_l1l1_ltheta.py:63-104 (per-row beta, learned per-row thresholds)
  V3  main_syn_l1l1_full.py:59-106   (per-row params, "VVar" E-step, beta3)
  V4  main_syn_l1l1_scalar.py:80-127 (scalar params, "VVar" E-step, beta3, returns T)
  V5  main_syn_l1l1_scalar_tied.py:82-129 (one shared fc scaled by ss1[k])
  V6  main_syn_lasso_scalar.py:65-114 (linear LASSO E-step)

and the per-layer training objectives of the reference training loops
  L1L1  main_syn_l1l1_scalar.py:290-294
  LASSO main_syn_lasso_scalar.py:276-281.

Pinned against the golden fixtures in tests/golden/*.npz, which were produced by running the
reference classes themselves (tests/golden/make_golden.py); see tests/test_oracle.py.
"""
from __future__ import annotations

import numpy as np

# thresholds of V1, plain tensors in the reference ctor (main_lena.py:40-41), not parameters
V1_THETA_Z = 0.025
V1_THETA_E = 0.06

# which reference variants return T (main_syn_l1l1_scalar.py:127) and which return (Z, E, L)
RETURNS_T = {"v1": False, "v2": False, "v3": False, "v4": True, "v5": True, "v6": True,
             "v7": False, "v7t": False, "v7p": False}


def self_active(x, theta):
    """relu(x - theta) - relu(-1.0 * x - theta)  (main_lena.py:52-53), literal two-relu form."""
    return np.maximum(x - theta, 0) - np.maximum(-1.0 * x - theta, 0)


_GEMM = None  # None: fp32 BLAS as the reference; "bf16" / "bf16_acc32": see _mm


def round_bf16(x):
    """fp32 -> bf16 -> fp32, round to nearest even (what the bf16 path feeds its MFMAs)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    r = ((u.astype(np.uint64) + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32).reshape(np.shape(x))


def _mm(a, b):
    """The GEMMs of the forward: fp32 (reference) or, for the bf16 operand mode of BASELINE
    config 5, both operands rounded to bf16 and the product accumulated in fp64, stored fp32
    ("bf16"), or accumulated in fp32 ("bf16_acc32": a second valid implementation of the same
    arithmetic, whose distance from "bf16" measures how far accumulation order alone moves the
    result -- the bf16 parity bar's yardstick d_k, tests/test_gpu_bf16.py)."""
    if _GEMM == "bf16":
        return (round_bf16(a).astype(np.float64) @ round_bf16(b).astype(np.float64)).astype(
            np.float32)
    if _GEMM == "bf16_acc32":
        return round_bf16(a) @ round_bf16(b)
    return a @ b


def _fc(W, Var):
    """nn.Linear(m, d, bias=False) applied as fc[k](Var.t()).t()  (main_lena.py:72)."""
    if _GEMM in ("bf16", "bf16_acc32"):
        return _mm(W, Var)
    return (Var.T @ W.T).T


def forward_news(variant, X, A, Z0, E0, L0, p, K, dtype):
    """The "new S" layer-wise schedule, forward(x, K) of main_syn_scalar_newS_layerwise.py:76-99
    (v7), main_syn_scalar_tied_newS_layerwise.py:76-99 (v7t, shared fc * ss1[k]) and
    main_syn_scalar_ptied_newS_layerwise.py:84-115 (v7p, fc[k // interval] * ss1[k])."""
    nfc = sum(1 for k in p if k.startswith("fc.") and k.endswith(".weight") and k != "fc.weight")
    total = sum(1 for k in p if k.startswith("beta1."))  # the model's layer count
    interval = max(total // nfc, 1) if variant == "v7p" else 1

    def fcW(k, Var):
        if variant == "v7":
            return _fc(p[f"fc.{k}.weight"], Var)
        W = p["fc.weight"] if variant == "v7t" else p[f"fc.{k // interval}.weight"]
        return p[f"ss1.{k}"] * _fc(W, Var)

    Z, E, L = [], [], []
    for k in range(K):
        if k == 0:
            E.append(E0)
            L.append(L0)
            Tn = _mm(A, Z0) + E0 - X
            Varn = L0 + p[f"beta1.{k}"] * Tn
            Z.append(self_active(Z0 - fcW(k, Varn), p[f"active_para.{k}"]))
        else:
            VVar = L[-1] + p[f"beta2.{k-1}"] * (_mm(A, Z[-1]) + E[-1] - X)
            E.append(self_active(E[-1] - p[f"ss2.{k-1}"] * VVar, p[f"active_para1.{k-1}"]))
            Tn = _mm(A, Z[-1]) + E[-1] - X
            L.append(L[-1] + p[f"beta3.{k-1}"] * Tn)
            Varn = L[-1] + p[f"beta1.{k}"] * Tn
            Z.append(self_active(Z[-1] - fcW(k, Varn), p[f"active_para.{k}"]))
    return dict(Z=Z, E=E, L=L)


def forward(variant, X, A, Z0, E0, L0, state_dict, layers, dtype=np.float32, gemm=None):
    """Run the reference forward of `variant` ('v1'..'v7p'); returns dict(Z, E, L[, T]) of lists.
    gemm="bf16" restates the bf16-operand mode (BASELINE config 5) instead of the reference's
    fp32 GEMMs ("bf16_acc32": the same with fp32 accumulation)."""
    global _GEMM
    prev, _GEMM = _GEMM, gemm
    try:
        return _forward(variant, X, A, Z0, E0, L0, state_dict, layers, dtype)
    finally:
        _GEMM = prev


def _forward(variant, X, A, Z0, E0, L0, state_dict, layers, dtype):
    c = lambda a: np.asarray(a, dtype=dtype)  # noqa: E731
    X, A, Z0, E0, L0 = c(X), c(A), c(Z0), c(E0), c(L0)
    p = {k: c(v) for k, v in state_dict.items()}
    if variant in ("v7", "v7t", "v7p"):
        return forward_news(variant, X, A, Z0, E0, L0, p, layers, dtype)
    T, Z, E, L = [], [], [], []
    for k in range(layers):
        if variant in ("v1", "v2"):
            # main_lena.py:68-89 (V1) / main_syn_l1l1_ltheta.py:59-80 (V2)
            b1, b2 = p[f"beta1.{k}"], p[f"beta2.{k}"]
            W = p[f"fc.{k}.weight"]
            if variant == "v1":
                thz, the = dtype(V1_THETA_Z), dtype(V1_THETA_E)
            else:
                thz, the = p[f"active_para.{k}"], p[f"active_para1.{k}"]
            Lp = L0 if k == 0 else L[-1]
            Zp = Z0 if k == 0 else Z[-1]
            if k == 0:
                T.append(_mm(A, Z0) + E0 - X)
            Var = Lp + b1 * T[-1]
            Z.append(self_active(Zp - _fc(W, Var), thz))
            E.append(self_active(X - _mm(A, Z[-1]) - b2 * Lp, the))
            T.append(_mm(A, Z[-1]) + E[-1] - X)
            L.append(Lp + b1 * T[-1])
        elif variant in ("v3", "v4", "v5"):
            # main_syn_l1l1_full.py:53-82 (V3), main_syn_l1l1_scalar.py:89-118 (V4),
            # main_syn_l1l1_scalar_tied.py:62-91 (V5)
            b1, b2, b3 = p[f"beta1.{k}"], p[f"beta2.{k}"], p[f"beta3.{k}"]
            ss2 = p[f"ss2.{k}"]
            thz, the = p[f"active_para.{k}"], p[f"active_para1.{k}"]
            Lp = L0 if k == 0 else L[-1]
            Zp = Z0 if k == 0 else Z[-1]
            Ep = E0 if k == 0 else E[-1]
            if k == 0:
                T.append(_mm(A, Z0) + E0 - X)
            Var = Lp + b1 * T[-1]
            if variant == "v5":
                Z.append(self_active(Zp - p[f"ss1.{k}"] * _fc(p["fc.weight"], Var), thz))
            else:
                Z.append(self_active(Zp - _fc(p[f"fc.{k}.weight"], Var), thz))
            VVar = Lp + b2 * (_mm(A, Z[-1]) + Ep - X)
            E.append(self_active(Ep - ss2 * VVar, the))
            T.append(_mm(A, Z[-1]) + E[-1] - X)
            L.append(Lp + b3 * T[-1])
        elif variant == "v6":
            # main_syn_lasso_scalar.py:74-107
            b1, b3 = p[f"beta1.{k}"], p[f"beta3.{k}"]
            s21, s22 = p[f"ss2_1.{k}"], p[f"ss2_2.{k}"]
            thz = p[f"active_para.{k}"]
            Lp = L0 if k == 0 else L[-1]
            Zp = Z0 if k == 0 else Z[-1]
            if k == 0:
                T.append(_mm(A, Z0) + E0 - X)
            Var = Lp + b1 * T[-1]
            Z.append(self_active(Zp - _fc(p[f"fc.{k}.weight"], Var), thz))
            residual = X - _mm(A, Z[-1])
            E.append(s21 * residual - s22 * Lp)
            T.append(_mm(A, Z[-1]) + E[-1] - X)
            L.append(Lp + b3 * T[-1])
        else:
            raise ValueError(f"unknown variant {variant!r}")
    out = dict(Z=Z, E=E, L=L)
    if RETURNS_T[variant]:
        out["T"] = T
    else:
        out["T_internal"] = T
    return out


def layer_objectives(Z, X, A, alpha, kind="l1l1"):
    """Per-layer objective the reference training loops log, averaged over the batch columns.

    l1l1:  alpha*sum(|Z_k|,0).mean() + sum(|X - A Z_k|,0).mean()        main_syn_l1l1_scalar.py:290-294
    lasso: alpha*sum(|Z_k|,0).mean() + 0.5*sum((X - A Z_k)^2,0).mean()  main_syn_lasso_scalar.py:276-281
    Accumulated in fp64 (the checker is the sum, not its rounding).
    """
    X = np.asarray(X, np.float64)
    A = np.asarray(A, np.float64)
    out = []
    for Zk in Z:
        Zk = np.asarray(Zk, np.float64)
        r = X - A @ Zk
        reg = alpha * np.abs(Zk).sum(0).mean()
        fit = np.abs(r).sum(0).mean() if kind == "l1l1" else 0.5 * (r ** 2).sum(0).mean()
        out.append(reg + fit)
    return np.array(out)


def nrel(a, b):
    """Norm-relative difference ||a - b||_F / ||b||_F (fp64)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
