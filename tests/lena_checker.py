"""Checker for the dual-gap training objective (test infrastructure): main_lena.py:221-228 with
dual_gap of :145-147 re-typed as torch ops, and the sign / start-layer of
main_syn_l1l1-dgap_ltheta.py:196-207.  Pinned to the reference scripts' own executed statements by
tests/test_oracle_lena.py (fixtures tests/golden/lena_*.npz, make_golden_lena.py)."""
import torch


def dual_gap(x, a):  # main_lena.py:145-147
    return torch.nn.functional.softplus(x - a) + torch.nn.functional.softplus(-x - a)


def lena_losses(Z, E, L, X, A, alpha, K, lx_sign=1.0, start=0):
    """One entry per layer (0.0 below `start`, as the dgap script's loop appends)."""
    out = []
    for k in range(K):
        if k < start:
            out.append(0.0)
            continue
        v = alpha * torch.mean(torch.abs(Z[k])) + torch.mean(torch.abs(E[k])) + \
            torch.mean(dual_gap(torch.mm(A.t(), L[k]), alpha)) + torch.mean(dual_gap(L[k], 1))
        out.append(v + torch.mean(L[k] * X) if lx_sign > 0 else v - torch.mean(L[k] * X))
    return out
