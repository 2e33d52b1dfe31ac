"""CPU restatement of the reference's classic KM / learned + safeguarded KM (LSKM) forward --
TEST INFRASTRUCTURE ONLY.

Only tests/ may import it, as the checker.  It restates, op for op in numpy, the test-script
class of /root/reference/test_syn_l1l1_scalar.py:

  KM(Zk, Ek, Lk, Tk, X)        :129-155  one LADMM step, beta = 1, ss1 = 0.999 / ||A^T A||_2,
                                         ss2 = 0.3, thresholds ss1*alpha and ss2
  S(Zk, Ek, Lk, Tk, X, Ep)     :158-175  fixed-point residual [beta Tn ; c (En - 2 Ek + Ep)]
  forward(x, use_learned, use_safeguard, continued, K)   :178-316
and the mu updaters of mu_updater.py:18-116 (EMA, GS, RT, None; RM is unusable in the reference:
its step returns torch's (values, indices) pair, which `(1.0-delta) * mu_k` cannot multiply).

Pinned against outputs of the reference class itself (tests/golden/make_golden_lskm.py ->
tests/golden/lskm_*.npz; tests/test_oracle_lskm.py).
"""
from __future__ import annotations

from math import sqrt

import numpy as np

from .dladmm_oracle import self_active


def lipschitz(A):
    """self.L = ||A^T A||_2 from the fp32 numpy copy of A (test_syn_l1l1_scalar.py:89), fp32."""
    A = np.asarray(A, np.float32)
    return np.float32(np.linalg.norm(np.matmul(A.T, A), ord=2))


class _Updater:
    """mu_updater.py: EMAUpdater (:18-32), GSUpdater (:34-52), RTUpdater (:55-73),
    BlankUpdater (:98-110)."""

    def __init__(self, method, mu, param):
        if method not in ("EMA", "GS", "RT", "None"):
            raise NotImplementedError(f"mu updater {method!r}")
        self.method, self.mu, self.p = method, mu, param

    def step(self, s_norm, keep):
        f = np.float32
        if self.method == "EMA":
            upd = f(self.p) * s_norm + f(1 - self.p) * self.mu
        elif self.method == "GS":
            upd = f(1 - self.p) * self.mu
        elif self.method == "RT":
            upd = s_norm
        else:
            self.mu = np.full_like(s_norm, 1e10)
            return self.mu
        self.mu = np.where(keep, upd, self.mu).astype(np.float32)
        return self.mu


def lskm_forward(X, A, Z0, E0, L0, sd, layers, use_learned, use_safeguard, continued, K, alpha,
                 delta=-99.0, mu_method="None", mu_param=0.0):
    """Returns dict(Z, E, L, T[, sg_count]) exactly as test_syn_l1l1_scalar.py:178-316."""
    f = np.float32
    X, A, Z0, E0, L0 = (np.asarray(a, f) for a in (X, A, Z0, E0, L0))
    p = {k: np.asarray(v, f) for k, v in sd.items()}
    Lc = lipschitz(A)
    ss1 = f(0.999) / Lc
    ss2 = f(0.3)
    beta = f(1.0)
    thz = ss1 * f(alpha)

    def km(Zk, Ek, Lk, Tk):
        Varn = Lk + beta * Tk
        Zn = self_active(Zk - ss1 * (A.T @ Varn), thz)
        TTn = A @ Zn + Ek - X
        En = self_active(Ek - ss2 * (Lk + beta * TTn), ss2)
        Tn = A @ Zn + En - X
        Ln = Lk + beta * Tn
        return Varn, Zn, En, Tn, Ln

    c = f(sqrt(0.3 / (1 - 0.3)))

    def s_norm(Zk, Ek, Lk, Tk, Ep):
        _, Zn, En, Tn, Ln = km(Zk, Ek, Lk, Tk)
        S = np.concatenate([beta * Tn, c * (En - f(2) * Ek + Ep)])
        return np.sqrt((S.astype(np.float64) ** 2).sum(0)).astype(f)

    T = [A @ Z0 + E0 - X]
    Z, E, L = [], [], []
    ret_cnt = use_learned and use_safeguard
    if ret_cnt:
        mu = s_norm(Z0, E0, L0, T[-1], E0)
        upd = _Updater(mu_method, mu, mu_param)
        sg = np.zeros(layers)
    for k in range(K):
        if continued and k == layers:
            use_learned = use_safeguard = False
        Zc = Z0 if k == 0 else Z[-1]
        Ec = E0 if k == 0 else E[-1]
        Lcur = L0 if k == 0 else L[-1]
        km_out = km(Zc, Ec, Lcur, T[-1])
        if use_learned:
            Var = Lcur + p[f"beta1.{k}"] * T[-1]
            Zl = self_active(Zc - (Var.T @ p[f"fc.{k}.weight"].T).T, p[f"active_para.{k}"])
            VV = Lcur + p[f"beta2.{k}"] * (A @ Zl + Ec - X)
            El = self_active(Ec - p[f"ss2.{k}"] * VV, p[f"active_para1.{k}"])
            Tl = A @ Zl + El - X
            Ll = Lcur + p[f"beta3.{k}"] * Tl
        if use_safeguard:
            nrm = s_norm(Zl, El, Ll, Tl, Ec)
            keep = nrm < f(1.0 - delta) * upd.mu
            upd.step(nrm, keep)
            sel = lambda a, b: np.where(keep[None, :], a, b)  # noqa: E731
            Z.append(sel(Zl, km_out[1]))
            E.append(sel(El, km_out[2]))
            T.append(sel(Tl, km_out[3]))
            L.append(sel(Ll, km_out[4]))
            sg[k] = float((~keep).sum())
        elif use_learned:
            Z.append(Zl); E.append(El); T.append(Tl); L.append(Ll)
        else:
            Z.append(km_out[1]); E.append(km_out[2]); T.append(km_out[3]); L.append(km_out[4])
    out = dict(Z=Z, E=E, L=L, T=T)
    if ret_cnt:
        out["sg_count"] = sg
    return out
