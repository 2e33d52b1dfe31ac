"""CPU restatement of the reference D-LADMM BACKWARD -- TEST INFRASTRUCTURE ONLY.

Parity oracle for SURVEY.md section 8 row f1 (backward through the fused op).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it, and only as the checker;
the product path never imports it.

The reference has no hand-written backward: its training loops (main_lena.py:216-233,
main_syn_l1l1_scalar.py:269-302, main_syn_lasso_scalar.py:258-290) call `total_loss.backward()`
and torch autograd differentiates the forward bodies of `DLADMMNet.forward`.  This module restates
that vector-Jacobian product by hand, as one reverse sweep over the layers, in numpy:

    forward(variant, ...)            the reference forward (dladmm_oracle.forward), keeping T
    vjp(variant, ..., gZ, gE, gL, gT) grads of sum_k <gZ_k,Z_k>+<gE_k,E_k>+<gL_k,L_k>+<gT_k,T_k>
                                      w.r.t. every state_dict entry (reference key names)
    train_loss_grads(...)             the upstream grads gZ_k of the reference training loss
                                      (main_syn_l1l1_scalar.py:283-298 / lasso :270-285)

Autograd conventions restated (torch 2.x CPU):
  relu'(v) = [v > 0]   (threshold_backward), so for S(x, th) = relu(x - th) - relu(-1.0*x - th)
                        (main_lena.py:52-53):  dS/dx = [x-th > 0] + [-x-th > 0],
                        dS/dth = -[x-th > 0] + [-x-th > 0]  (both evaluated in the forward dtype)
  |v|'   = sgn(v)       (sgn(0) = 0)
  broadcast params receive the sum of their element grads over the broadcast axes.

Pinned against gradients produced by the reference classes themselves under torch autograd
(tests/golden/make_golden_grad.py -> tests/golden/grad_*.npz; tests/test_oracle_grad.py).
"""
from __future__ import annotations

import numpy as np

from .dladmm_oracle import V1_THETA_E, V1_THETA_Z, self_active

EM_V1, EM_VVAR, EM_LASSO = 0, 1, 2


def _layer_params(variant, p, k, dtype, interval=1):
    """Per-layer parameters in the normalised form of the fused kernel (include/dladmm.h slots),
    plus, per slot, the state_dict key it came from (None = not a parameter).  The newS
    schedules (v7, v7t, v7p) have V4's / V5's per-layer algebra (see vjp)."""
    if variant == "v7":
        variant = "v4"
    if variant == "v7t":
        variant = "v5"
    if variant == "v7p":
        q, keys = _layer_params("v5", dict(p, **{"fc.weight": p[f"fc.{k // interval}.weight"]}),
                                k, dtype)
        keys["W"] = f"fc.{k // interval}.weight"
        return q, keys
    if variant in ("v1", "v2"):
        # main_lena.py:84-89: b1 serves Var and L (beta1), b2 the E-step; V1 thetas are constants
        q = dict(b1=p[f"beta1.{k}"], b2=p[f"beta2.{k}"], b3=p[f"beta1.{k}"],
                 W=p[f"fc.{k}.weight"], s1=dtype(1.0), em=EM_V1)
        keys = dict(b1=f"beta1.{k}", b2=f"beta2.{k}", b3=f"beta1.{k}", W=f"fc.{k}.weight")
        if variant == "v1":
            q.update(thz=dtype(V1_THETA_Z), the=dtype(V1_THETA_E))
        else:
            q.update(thz=p[f"active_para.{k}"], the=p[f"active_para1.{k}"])
            keys.update(thz=f"active_para.{k}", the=f"active_para1.{k}")
        return q, keys
    if variant in ("v3", "v4", "v5"):
        q = dict(b1=p[f"beta1.{k}"], b2=p[f"beta2.{k}"], b3=p[f"beta3.{k}"], ss2=p[f"ss2.{k}"],
                 thz=p[f"active_para.{k}"], the=p[f"active_para1.{k}"], em=EM_VVAR)
        keys = dict(b1=f"beta1.{k}", b2=f"beta2.{k}", b3=f"beta3.{k}", ss2=f"ss2.{k}",
                    thz=f"active_para.{k}", the=f"active_para1.{k}")
        if variant == "v5":
            q.update(W=p["fc.weight"], s1=p[f"ss1.{k}"])
            keys.update(W="fc.weight", s1=f"ss1.{k}")
        else:
            q.update(W=p[f"fc.{k}.weight"], s1=None)
            keys.update(W=f"fc.{k}.weight")
        return q, keys
    if variant == "v6":
        q = dict(b1=p[f"beta1.{k}"], b3=p[f"beta3.{k}"], ss2=p[f"ss2_1.{k}"],
                 ss2b=p[f"ss2_2.{k}"], thz=p[f"active_para.{k}"], W=p[f"fc.{k}.weight"],
                 s1=None, em=EM_LASSO)
        keys = dict(b1=f"beta1.{k}", b3=f"beta3.{k}", ss2=f"ss2_1.{k}", ss2b=f"ss2_2.{k}",
                    thz=f"active_para.{k}", W=f"fc.{k}.weight")
        return q, keys
    raise ValueError(f"unknown variant {variant!r}")


def _shrink_d(x, th):
    """(dS/dx, dS/dth) of the literal two-relu shrink, torch's relu' = [v > 0]."""
    a = (x - th) > 0
    b = (-1.0 * x - th) > 0
    return a.astype(x.dtype) + b.astype(x.dtype), b.astype(x.dtype) - a.astype(x.dtype)


def _reduce_to(g, shape):
    """Sum a full (rows, B) grad down to a broadcast param's shape ((rows,1), (1,1), (rows,B))."""
    g = np.asarray(g)
    if tuple(shape) == g.shape:
        return g
    if len(shape) == 2 and shape[1] == 1 and shape[0] == g.shape[0]:
        return g.sum(axis=1, keepdims=True)
    return np.array(g.sum(), dtype=g.dtype).reshape(shape)


def vjp(variant, X, A, Z0, E0, L0, state_dict, layers, gZ=None, gE=None, gL=None, gT=None,
        dtype=np.float32):
    """Gradient of sum_k <gZ[k],Z_k> + <gE[k],E_k> + <gL[k],L_k> + sum_j <gT[j],T_j> w.r.t. every
    entry of `state_dict` (same keys; None-grads come back as zeros).  gZ/gE/gL: K arrays or None,
    gT: K+1 arrays or None.  The forward is recomputed here in `dtype`, op for op as the
    reference (dladmm_oracle.forward), and the reverse sweep follows it in reverse."""
    c = lambda a: np.asarray(a, dtype=dtype)  # noqa: E731
    X, A, Z0, E0, L0 = c(X), c(A), c(Z0), c(E0), c(L0)
    p = {k: c(v) for k, v in state_dict.items()}
    K = layers
    interval = 1
    if variant in ("v7", "v7t", "v7p"):
        # newS (main_syn_scalar_newS_layerwise.py:76-99): Z[k] = V4 Z_k, E[k] = V4 E_{k-1}
        # (E[0] = E0), L[k] = V4 L_{k-1}; the V4 sweep with the E/L cotangents shifted by one
        # layer (E[0], L[0] are inputs; V4's last E_{K-1}, L_{K-1}, T_K are never outputs)
        shift = lambda seq: None if seq is None else [c(g) for g in seq[1:]] + [None]  # noqa
        gE, gL, gT = shift(gE), shift(gL), None
        if variant == "v7p":
            nfc = sum(1 for k in p if k.startswith("fc.") and k.endswith(".weight"))
            interval = max(sum(1 for k in p if k.startswith("beta1.")) // nfc, 1)
    # ---- forward, keeping every intermediate the reverse sweep needs
    Zs, Es, Ls, Ts, Vs, Us, Ps, Qs, Eh = [Z0], [E0], [L0], [A @ Z0 + E0 - X], [], [], [], [], []
    prm = []
    for k in range(K):
        q, keys = _layer_params(variant, p, k, dtype, interval)
        prm.append((q, keys))
        Zp, Ep, Lp = Zs[-1], Es[-1], Ls[-1]
        Var = Lp + q["b1"] * Ts[-1]
        Q = (Var.T @ q["W"].T).T                       # fc[k](Var.t()).t()
        U = Zp - (Q if q["s1"] is None else q["s1"] * Q)
        Z = self_active(U, q["thz"])
        P = A @ Z
        if q["em"] == EM_V1:
            eh = X - P - q["b2"] * Lp                  # main_lena.py:87
            E = self_active(eh, q["the"])
        elif q["em"] == EM_VVAR:
            VV = Lp + q["b2"] * (P + Ep - X)           # main_syn_l1l1_scalar.py:114
            eh = Ep - q["ss2"] * VV                    # :115
            E = self_active(eh, q["the"])
        else:
            eh = None
            E = q["ss2"] * (X - P) - q["ss2b"] * Lp    # main_syn_lasso_scalar.py:102-103
        T = P + E - X
        L = Lp + q["b3"] * T
        Vs.append(Var); Us.append(U); Ps.append(P); Qs.append(Q); Eh.append(eh)
        Zs.append(Z); Es.append(E); Ls.append(L); Ts.append(T)

    zero_n = np.zeros_like(Z0)
    zero_m = np.zeros_like(X)
    up = lambda seq, i, z: z if seq is None or seq[i] is None else c(seq[i])  # noqa: E731
    grads = {k: np.zeros_like(v) for k, v in p.items()}

    def acc(key, g):
        if key is not None:
            grads[key] = grads[key] + _reduce_to(g, grads[key].shape).astype(dtype)

    # adjoints carried from layer k+1 into layer k (of Z_k, E_k, L_k, T_{k+1})
    aZ, aE, aL, aT = zero_n, zero_m, zero_m, zero_m
    for k in reversed(range(K)):
        q, keys = prm[k]
        Zp, Ep, Lp, Tk = Zs[k], Es[k], Ls[k], Ts[k]
        Var, U, P, Q = Vs[k], Us[k], Ps[k], Qs[k]
        aZ = aZ + up(gZ, k, zero_n)
        aE = aE + up(gE, k, zero_m)
        aL = aL + up(gL, k, zero_m)
        aT = aT + up(gT, k + 1, zero_m)
        # L_k = Lp + b3 * T_{k+1}
        gTn = aT + q["b3"] * aL
        acc(keys.get("b3"), aL * Ts[k + 1])
        gLp = aL
        # T_{k+1} = P + E_k - X
        gEt = aE + gTn
        gP = gTn
        gEp = zero_m
        if q["em"] == EM_V1:
            dx, dth = _shrink_d(Eh[k], q["the"])
            gEh = gEt * dx
            acc(keys.get("the"), gEt * dth)
            gP = gP - gEh
            acc(keys.get("b2"), -gEh * Lp)
            gLp = gLp - q["b2"] * gEh
        elif q["em"] == EM_VVAR:
            dx, dth = _shrink_d(Eh[k], q["the"])
            gEh = gEt * dx
            acc(keys.get("the"), gEt * dth)
            VV = Lp + q["b2"] * (P + Ep - X)
            gEp = gEh
            gVV = -q["ss2"] * gEh
            acc(keys.get("ss2"), -gEh * VV)
            gLp = gLp + gVV
            acc(keys.get("b2"), gVV * (P + Ep - X))
            gP = gP + q["b2"] * gVV
            gEp = gEp + q["b2"] * gVV
        else:
            acc(keys.get("ss2"), gEt * (X - P))
            gP = gP - q["ss2"] * gEt
            acc(keys.get("ss2b"), -gEt * Lp)
            gLp = gLp - q["ss2b"] * gEt
        # P = A Z_k
        gZt = aZ + A.T @ gP
        # Z_k = S(U, thz)
        dx, dth = _shrink_d(U, q["thz"])
        gU = gZt * dx
        acc(keys.get("thz"), gZt * dth)
        # U = Zp - s1 * Q, Q = W Var
        s1 = dtype(1.0) if q["s1"] is None else q["s1"]
        acc(keys.get("s1"), -gU * Q)
        gQ = -s1 * gU
        acc(keys["W"], gQ @ Var.T)
        gVar = q["W"].T @ gQ
        # Var = Lp + b1 * T_k
        gLp = gLp + gVar
        acc(keys.get("b1"), gVar * Tk)
        aZ, aE, aL, aT = gU, gEp, gLp, q["b1"] * gVar
    return grads


def train_loss_grads(Z, X, A, alpha, coeffs, kind="l1l1", dtype=np.float32):
    """Upstream grads d(total_loss)/dZ_k of the reference training loss
        total = sum_k coeffs[k] * (alpha*sum(|Z_k|,0).mean() + sum(|X - A Z_k|,0).mean())  (l1l1,
        main_syn_l1l1_scalar.py:283-298) or with 0.5*sum((X - A Z_k)^2,0).mean() (lasso,
        main_syn_lasso_scalar.py:270-285), where coeffs[k] = decay (0.6**epoch, 1 for the last)."""
    X = np.asarray(X, dtype)
    A = np.asarray(A, dtype)
    B = X.shape[1]
    out = []
    for k, Zk in enumerate(Z):
        Zk = np.asarray(Zk, dtype)
        r = X - A @ Zk
        g_r = np.sign(r) if kind == "l1l1" else r
        g = dtype(coeffs[k]) * (dtype(alpha) / dtype(B) * np.sign(Zk) - (A.T @ g_r) / dtype(B))
        out.append(g.astype(dtype))
    return out
