"""Torch-op CPU restatement of the reference forward -- TEST INFRASTRUCTURE / CPU BASELINE ONLY.

Only tests/ and bench.py's `cpu_baseline` leg import this module: it is the CPU baseline the
bench times (BASELINE.md "CPU baseline": the reference op sequence in torch, fp32, no_grad, on the
cores the GPU box grants) and it is pinned to the golden fixtures the reference classes produced
(tests/test_oracle_torch.py).  The product path (d-ladmm_amd/) never imports it.

It issues the reference's ATen ops in the reference's order -- including the duplicated
`A.mm(Z_k)` of every layer and `fc[k](Var.t()).t()` as a bias-free linear on the transposed
operand -- so its time is the reference's CPU time:

  V1  main_lena.py:57-98              E = S((X - A.mm(Z)) - b2.mul(L), 0.06), L += b1.mul(T)
  V2  main_syn_l1l1_ltheta.py:63-104  V1 with per-row parameters
  V3  main_syn_l1l1_full.py:59-106    VVar E-step, beta3, per-row parameters
  V4  main_syn_l1l1_scalar.py:80-127  VVar E-step, beta3, scalar parameters, returns T
  V5  main_syn_l1l1_scalar_tied.py:82-129  Z = S(Z - ss1[k] * fc(Var.t()).t())
  V6  main_syn_lasso_scalar.py:65-114 E = ss2_1.mul(X - A.mm(Z)) - ss2_2.mul(L)
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

V1_THETA = (0.025, 0.06)  # main_lena.py:40-41 (plain tensors, not parameters)


def _shrink(x, th):
    """F.relu(x - th) - F.relu(-1.0 * x - th)  (main_lena.py:52-53)."""
    return F.relu(x - th) - F.relu(-1.0 * x - th)


def _linear(W, Var):
    """fc[k](Var.t()).t() with nn.Linear(m, d, bias=False): weight W is (d, m)  (main_lena.py:72)."""
    return F.linear(Var.t(), W).t()


@torch.no_grad()
def forward(variant, X, A, Z0, E0, L0, params, layers):
    """The reference forward of `variant` (v1..v6) on torch CPU tensors; `params` maps the
    reference state_dict keys to tensors.  Returns (Z, E, L[, T]) lists like the reference."""
    p = dict(params)
    # the reference builds every fc weight as Parameter(A.t() + 1e-3 * randn_like(A.t())) (* 0.4)
    # (main_lena.py:49, main_syn_l1l1_scalar.py:72): elementwise ops on the transposed view keep
    # its strides, so the weight is (d, m) in column-major layout, and load_state_dict copies into
    # that storage.  F.linear then runs the GEMM with the transposed-weight operand; keep the
    # layout so the same BLAS kernel (and summation order) runs
    for key in [k for k in p if k.startswith("fc.")]:
        p[key] = p[key].t().contiguous().t()
    if variant == "v1":
        thz = torch.tensor(V1_THETA[0], dtype=torch.float32)
        the = torch.tensor(V1_THETA[1], dtype=torch.float32)
    T, Z, E, L = [], [], [], []
    for k in range(layers):
        Zp = Z0 if k == 0 else Z[-1]
        Ep = E0 if k == 0 else E[-1]
        Lp = L0 if k == 0 else L[-1]
        if k == 0:
            T.append(A.mm(Z0) + E0 - X)
        # Step 1: Var and the Z update
        Var = Lp + p[f"beta1.{k}"].mul(T[-1])
        if variant != "v1":
            thz = p[f"active_para.{k}"]
        if variant == "v5":
            Z.append(_shrink(Zp - p[f"ss1.{k}"] * _linear(p["fc.weight"], Var), thz))
        else:
            Z.append(_shrink(Zp - _linear(p[f"fc.{k}.weight"], Var), thz))
        # Step 2: the E update (one A.mm(Z_k) of the two the reference forms per layer)
        if variant in ("v1", "v2"):
            if variant == "v2":
                the = p[f"active_para1.{k}"]
            E.append(_shrink(X - A.mm(Z[-1]) - p[f"beta2.{k}"].mul(Lp), the))
        elif variant in ("v3", "v4", "v5"):
            VVar = Lp + p[f"beta2.{k}"] * (A.mm(Z[-1]) + Ep - X)
            E.append(_shrink(Ep - p[f"ss2.{k}"].mul(VVar), p[f"active_para1.{k}"]))
        elif variant == "v6":
            residual = X - A.mm(Z[-1])
            E.append(p[f"ss2_1.{k}"].mul(residual) - p[f"ss2_2.{k}"].mul(Lp))
        else:
            raise ValueError(f"unknown variant {variant!r}")
        # Step 3: the residual (the second A.mm(Z_k)) and the dual
        T.append(A.mm(Z[-1]) + E[-1] - X)
        b3 = p[f"beta1.{k}"] if variant in ("v1", "v2") else p[f"beta3.{k}"]
        L.append(Lp + b3.mul(T[-1]))
    if variant in ("v4", "v5", "v6"):
        return Z, E, L, T
    return Z, E, L
