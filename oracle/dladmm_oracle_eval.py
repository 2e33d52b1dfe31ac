"""CPU restatement of the reference test scripts' evaluation objectives -- TEST INFRASTRUCTURE
ONLY.  Only tests/ may import it, as the checker.

Each function restates, in numpy fp64, the per-batch accumulation of one objective of
/root/reference/test_syn_l1l1_scalar.py:436-489 (and test_syn_lasso_scalar.py:477-503), literally
with the product A @ Z_k, and returns the per-layer batch sums the reference adds into its
accumulators.  Pinned: tests/test_oracle_eval.py checks every function against fixtures that
EXECUTED the reference scripts' own objective statements (tests/golden/make_golden_eval.py:
test_syn_l1l1_scalar.py:450-604 and test_syn_lasso_scalar.py:446-568, ast-extracted and run on
the scripts' own model class), tests/golden/eval_*.npz.
"""
from __future__ import annotations

import numpy as np


def _f(a):
    return np.asarray(a, np.float64)


def nmse_terms(Z, E, Zl, El):
    """(sum (Z* - Z_k)^2, sum (E* - E_k)^2) per layer   (:440-442)."""
    return (np.array([((_f(Zl) - _f(z)) ** 2).sum() for z in Z]),
            np.array([((_f(El) - _f(e)) ** 2).sum() for e in E]))


def l1l1(Z, X, A, alpha):
    """alpha sum|Z_k| + sum|X - A Z_k|   (:444-448)."""
    return np.array([alpha * np.abs(_f(z)).sum() + np.abs(_f(X) - _f(A) @ _f(z)).sum() for z in Z])


def lasso(Z, X, A, alpha, per_sample=False):
    """alpha sum|Z_k| + 0.5 sum (X - A Z_k)^2   (test_syn_lasso_scalar.py:491-503)."""
    v = [alpha * np.abs(_f(z)).sum(0) + 0.5 * ((_f(X) - _f(A) @ _f(z)) ** 2).sum(0) for z in Z]
    return np.stack(v, 1) if per_sample else np.array([x.sum() for x in v])


def normalized_l1l1(Z, X, A, alpha, Zgt):
    """sum_b |l1l1_b(Z_k) - l1l1_b(Zgt)| / l1l1_b(Zgt)   (:450-462)."""
    col = lambda z: alpha * np.abs(_f(z)).sum(0) + np.abs(_f(X) - _f(A) @ _f(z)).sum(0)  # noqa
    g = col(Zgt)
    return np.array([(np.abs(col(z) - g) / g).sum() for z in Z])


def gt(Z, E, Zgt, Egt):
    """sum (Z_k - Zgt)^2 + sum (E_k - Egt)^2   (:464-468)."""
    return np.array([((_f(z) - _f(Zgt)) ** 2).sum() + ((_f(e) - _f(Egt)) ** 2).sum()
                     for z, e in zip(Z, E)])


def normalized_gt(Z, E, Zgt, Egt):
    """sum_b (|Z_k - Zgt|_b^2 + |E_k - Egt|_b^2) / (|Zgt|_b^2 + |Egt|_b^2)   (:470-479)."""
    den = (_f(Zgt) ** 2).sum(0) + (_f(Egt) ** 2).sum(0)
    return np.array([((((_f(z) - _f(Zgt)) ** 2).sum(0) + ((_f(e) - _f(Egt)) ** 2).sum(0)) / den)
                     .sum() for z, e in zip(Z, E)])


def s_l2(Z, E, L, T, X, A, E0, alpha, Lc):
    """sum_b |S(Z_k, E_k, L_k, T_{k+1}, X, E_{k-1})|_b with the KM constants of :158-175
    (beta = 1, ss1 = 0.999 / Lc, ss2 = 0.3)   (:481-486)."""
    from .dladmm_oracle import self_active
    A, X = _f(A), _f(X)
    ss1, ss2, c = 0.999 / float(Lc), 0.3, np.sqrt(0.3 / 0.7)
    out = []
    for k in range(len(Z)):
        Zk, Ek, Lk, Tk = _f(Z[k]), _f(E[k]), _f(L[k]), _f(T[k + 1])
        Ep = _f(E0) if k == 0 else _f(E[k - 1])
        Var = Lk + Tk
        Zn = self_active(Zk - ss1 * (A.T @ Var), ss1 * alpha)
        En = self_active(Ek - ss2 * (Lk + (A @ Zn + Ek - X)), ss2)
        Tn = A @ Zn + En - X
        S = np.concatenate([Tn, c * (En - 2 * Ek + Ep)])
        out.append(np.sqrt((S ** 2).sum(0)).sum())
    return np.array(out)
