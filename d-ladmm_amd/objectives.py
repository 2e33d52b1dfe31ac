"""Evaluation objectives of the reference test scripts, reduced from
per-column values computed on the GPU instead of K extra products A Z_k per batch.

The reference accumulates, batch by batch over the test set, one of
  NMSE             sum (Z* - Z_k)^2, sum (E* - E_k)^2 -> 10 log10(mse_z/|Z*|^2 + mse_e/|E*|^2)
                   (test_syn_l1l1_scalar.py:440-442, :507-522)
  L1L1             alpha sum|Z_k| + sum|X - A Z_k|                     (:444-448, :524-530)
  LASSO            alpha sum|Z_k| + 0.5 sum (X - A Z_k)^2       (test_syn_lasso_scalar.py:491-495)
  LASSO-ALL        the same per sample                                  (:496-503)
  Normalized-L1L1  sum_b |l1l1_b(Z_k) - l1l1_b(Zgt)| / l1l1_b(Zgt)      (:450-462)
  GT               sum (Z_k - Zgt)^2 + sum (E_k - Egt)^2                (:464-468)
  Normalized-GT    sum_b (|Z_k - Zgt|_b^2 + |E_k - Egt|_b^2) / (|Zgt|_b^2 + |Egt|_b^2) (:470-479)
  S-L2             sum_b |S(Z_k, E_k, L_k, T_{k+1}, X, E_{k-1})|_b                (:481-486)
where (Zgt, Egt) is the last iterate of a long classic KM run (the scripts use K = 2000).

Per-column sums come from `dladmm_colobj_f32` (csrc/dladmm_eval.hip), which reads X - A Z_k as
E_k - T_{k+1} (the identity T_{k+1} = A Z_k + E_k - X of main_lena.py:88); S-L2 runs ONE KM step
over all K layers at once (the layers stacked along the batch, columns being independent) and
the safeguard kernel's norm.

Parity (tests/test_gpu_eval.py) is pinned by fixtures that executed the reference scripts' own
objective statements (tests/golden/make_golden_eval.py, eval_*.npz): on the reference forward's
outputs (the objective computation alone, 1e-5) and end to end (forward + K = 2000 KM ground
truth + objectives on the GPU, 1e-4).
"""
from __future__ import annotations

import ctypes
from math import sqrt
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib

OBJECTIVES = ("NMSE", "L1L1", "LASSO", "LASSO-ALL", "Normalized-L1L1", "GT", "Normalized-GT",
              "S-L2")


def _stack(seq: Sequence[torch.Tensor]):
    """(base tensor, layer stride, row stride) when the layers are equally spaced views of one
    allocation (what every forward here returns), else None."""
    if len(seq) == 0:
        return None
    ld = seq[0].stride(0)
    if any(t.stride(0) != ld or t.stride(1) != 1 for t in seq):
        return None
    if len(seq) == 1:
        return seq[0], 0, ld
    step = seq[1].data_ptr() - seq[0].data_ptr()
    for k in range(len(seq)):
        if seq[k].data_ptr() != seq[0].data_ptr() + k * step:
            return None
    return seq[0], step // 4, ld


def column_terms(Z, E=None, T=None, Zref=None, Eref=None, fit_kind: str = "l1l1",
                 want=("reg", "fit", "dz", "de")):
    """Per-layer, per-column sums as fp64 [K, B] tensors (dict): reg = sum|Z_k|, fit =
    sum|E_k - T_{k+1}| (or 0.5 sum of squares for 'lasso'), dz = sum (Zref - Z_k)^2,
    de = sum (Eref - E_k)^2.  Z, E: K tensors (rows, B); T: K+1 tensors."""
    L = _lib.lib()
    K = len(Z)
    n, B = Z[0].shape
    dev = Z[0].device
    m = E[0].shape[0] if E is not None else 1
    out = {w: torch.empty((K, B), device=dev, dtype=torch.float64) for w in want}
    groups = [(0, K)]
    # T: exactly the views the launch below reads (T_0 .. T_K: layer k reads T_{k+1} at one
    # layer stride from T_0), not just T_1.. -- separately allocated tensors may happen to be
    # equally spaced from T_1 on while T_0 is not
    stacks = [_stack(Z), _stack(E) if E is not None else (None, 0, 0),
              _stack(T[:K + 1]) if T is not None else (None, 0, 0)]
    if any(s is None for s in stacks):
        groups = [(k, k + 1) for k in range(K)]   # not one allocation: one launch per layer
    stream = torch.cuda.current_stream(dev).cuda_stream
    for k0, k1 in groups:
        d = _lib.ColObjDesc()
        d.abi_version = _lib.ABI_VERSION
        d.m, d.n, d.batch, d.layers = m, n, B, k1 - k0
        d.fit_kind = _lib.LOSS_LASSO if fit_kind == "lasso" else _lib.LOSS_L1L1
        zs = _stack(Z[k0:k1])
        d.Z, d.z_layer_stride, d.ld_z = zs[0].data_ptr(), zs[1], zs[2]
        if E is not None:
            es = _stack(E[k0:k1])
            d.E, d.e_layer_stride, d.ld_e = es[0].data_ptr(), es[1], es[2]
        if T is not None:
            ts = _stack(T[k0:k1 + 1])
            d.T, d.t_layer_stride, d.ld_t = ts[0].data_ptr(), ts[1], ts[2]
        if Zref is not None:
            d.Zref, d.ld_zref = Zref.data_ptr(), Zref.stride(0)
        if Eref is not None:
            d.Eref, d.ld_eref = Eref.data_ptr(), Eref.stride(0)
        for w in want:
            setattr(d, w, out[w][k0:k1].data_ptr())
        _lib.check(L.dladmm_colobj_f32(ctypes.byref(d), ctypes.c_void_p(stream)))
    return out


def s_norms(model, X, Z, E, L, E0):
    """|S(Z_k, E_k, L_k, T_{k+1}, X, E_{k-1})| per layer and column (test_syn_l1l1_scalar.py:
    481-486) for a DLADMMNetLSKM-like `model`: one KM step over the K layers stacked along the
    batch, then the safeguard kernel's residual norm.  Returns fp32 [K, B]."""
    K = len(Z)
    B = X.shape[1]
    Zs = torch.cat(list(Z), 1)
    Es = torch.cat(list(E), 1)
    Ls = torch.cat(list(L), 1)
    Xs = X.repeat(1, K)
    Ep = torch.cat([E0] + list(E[:-1]), 1)
    step = model._km(Xs, Zs, Es, Ls, 1)
    mu = torch.empty(K * B, device=X.device, dtype=torch.float32)
    lib = _lib.lib()
    d = _lib.SafeguardDesc()
    d.abi_version = _lib.ABI_VERSION
    d.m, d.n, d.batch, d.ld = X.shape[0], Z[0].shape[0], K * B, K * B
    d.Es, d.Ts, d.El, d.Ep, d.mu = (step.E[0].data_ptr(), step.T[1].data_ptr(), Es.data_ptr(),
                                    Ep.data_ptr(), mu.data_ptr())
    d.beta, d.c, d.delta, d.updater = 1.0, sqrt(0.3 / (1 - 0.3)), 0.0, _lib.MU_NONE
    stream = torch.cuda.current_stream(X.device).cuda_stream
    _lib.check(lib.dladmm_safeguard_f32(ctypes.byref(d), ctypes.c_void_p(stream)))
    return mu.reshape(K, B)


class Evaluator:
    """Accumulates one of OBJECTIVES over test batches exactly as the reference test loop does
    and finalises it (`result`).  `add_batch` takes the forward's lists (Z, E, L, T) of one batch
    plus, as the objective needs, the labels (Z*, E*), the ground truth (Zgt, Egt, Tgt: the last
    iterate of a long KM run on the same batch) or the model (S-L2)."""

    def __init__(self, objective: str, K: int, alpha: float, n_test: Optional[int] = None):
        if objective not in OBJECTIVES:
            raise NotImplementedError(f"objective `{objective}` not supported")
        self.objective, self.K, self.alpha = objective, K, float(alpha)
        self.n_test = n_test
        self.acc = np.zeros(K)
        self.acc_e = np.zeros(K)
        self.all = []   # LASSO-ALL per-sample rows

    def add_batch(self, X, Z, E, L=None, T=None, Z_label=None, E_label=None, gt=None,
                  model=None):
        K, ob = self.K, self.objective
        Z, E = list(Z)[:K], list(E)[:K]
        if ob == "NMSE":
            c = column_terms(Z, E, None, Z_label, E_label, want=("dz", "de"))
            self.acc += c["dz"].sum(1).cpu().numpy()
            self.acc_e += c["de"].sum(1).cpu().numpy()
        elif ob in ("L1L1", "LASSO", "LASSO-ALL"):
            c = column_terms(Z, E, list(T)[:K + 1], fit_kind="l1l1" if ob == "L1L1" else "lasso",
                             want=("reg", "fit"))
            v = self.alpha * c["reg"] + c["fit"]
            if ob == "LASSO-ALL":
                self.all.append(v.t().cpu().numpy())
            else:
                self.acc += v.sum(1).cpu().numpy()
        elif ob == "Normalized-L1L1":
            Zg, Eg, Tg = gt
            c = column_terms(Z, E, list(T)[:K + 1], want=("reg", "fit"))
            g = column_terms([Zg], [Eg], [Tg, Tg], want=("reg", "fit"))
            gv = self.alpha * g["reg"] + g["fit"]                     # [1, B]
            v = self.alpha * c["reg"] + c["fit"]
            self.acc += ((v - gv).abs() / gv).sum(1).cpu().numpy()
        elif ob in ("GT", "Normalized-GT"):
            Zg, Eg = gt[0], gt[1]
            c = column_terms(Z, E, None, Zg, Eg, want=("dz", "de"))
            if ob == "GT":
                self.acc += (c["dz"] + c["de"]).sum(1).cpu().numpy()
            else:
                nrm = column_terms([Zg], [Eg], None, torch.zeros_like(Zg), torch.zeros_like(Eg),
                                   want=("dz", "de"))
                den = nrm["dz"] + nrm["de"]
                self.acc += ((c["dz"] + c["de"]) / den).sum(1).cpu().numpy()
        else:  # S-L2
            s = s_norms(model, X, Z, E, list(L)[:K], model.E0)
            self.acc += s.double().sum(1).cpu().numpy()

    def result(self, Z_ts=None, E_ts=None):
        """Finalised per-layer values (test_syn_l1l1_scalar.py:507-595)."""
        ob, n = self.objective, self.n_test
        if ob == "NMSE":
            dz = float((np.asarray(Z_ts, np.float64) ** 2).sum()) / n
            de = float((np.asarray(E_ts, np.float64) ** 2).sum()) / n
            return 10 * np.log10(self.acc / n / dz + self.acc_e / n / de)
        if ob == "LASSO-ALL":
            return np.concatenate(self.all, 0)
        return self.acc / n
