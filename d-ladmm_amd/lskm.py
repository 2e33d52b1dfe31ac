"""Classic KM (LADMM) iteration and learned + safeguarded KM (LSKM): the test-script model of
/root/reference/test_syn_l1l1_scalar.py:73-322 as a drop-in.

Same constructor and parameters as the V4 model (its `state_dict` loads unchanged), plus the
settings the reference reads from module globals (alpha, delta, mu_k_method, mu_k_param,
num_iter) as keyword arguments.  `forward(x, use_learned, use_safeguard, continued, K)` returns
(Z, E, L, T) or, with learned + safeguard, (Z, E, L, T, sg_count) like the reference.

Every step runs on the HIP kernels:
  * a KM step is the fused K-layer kernel's V5 path with the shared weight A^T, step
    ss1 = 0.999 / ||A^T A||_2, thresholds ss1*alpha and ss2 = 0.3, beta = 1 -- operation for
    operation the reference's KM (:129-155).  A pure KM run of K iterations (the K = 2000 ground
    truth of the test scripts) is ONE kernel launch with the weight packed once;
  * a learned step is the V4 path on layer k's parameters;
  * the safeguard (fixed-point residual norm, mu update, per-column select) is
    `dladmm_safeguard_f32` (csrc/dladmm_lskm.hip).
"""
from __future__ import annotations

import ctypes
from math import sqrt
from typing import Optional

import numpy as np
import torch

from . import _lib
from .model import DLADMMNetScalar, _scalar_table
from .ops import dladmm_forward

_UPDATERS = {"None": _lib.MU_NONE, "EMA": _lib.MU_EMA, "GS": _lib.MU_GS, "RT": _lib.MU_RT}


class DLADMMNetLSKM(DLADMMNetScalar):
    """test_syn_l1l1_scalar.py:73-322 (also the LSKM classes of test_syn_l1l1_newS*.py /
    test_syn_scalar_*_Acols.py share this KM / S / safeguard machinery)."""
    WSCALE = 1.0   # :113: m.weight = A.t() + 1e-3 * randn (no 0.4)
    NAME = "DLADMMNet"

    def __init__(self, m, n, d, batch_size, A, Z0, E0, L0, layers, *, alpha: float = 0.01,
                 delta: float = -99.0, mu_k_method: str = "None", mu_k_param: float = 0.0,
                 num_iter: int = 200):
        super().__init__(m, n, d, batch_size, A, Z0, E0, L0, layers)
        if mu_k_method == "RM":
            raise NotImplementedError(
                "mu_k_method 'RM': the reference RMUpdater.step returns torch's (values, indices) "
                "pair (mu_updater.py:94), which test_syn_l1l1_scalar.py:232 cannot multiply")
        if mu_k_method not in _UPDATERS:
            raise ValueError(f"unknown mu_k_method {mu_k_method!r}")
        # the reference's module globals (test_syn_l1l1_scalar.py:39-50)
        self.alpha, self.delta = float(alpha), float(delta)
        self.mu_k_method, self.mu_k_param = mu_k_method, float(mu_k_param)
        self.num_iter = int(num_iter)

    # --- the KM step's constants (:129-132): beta = 1, ss1 = 0.999 / L, ss2 = 0.3 -------------
    def _km_table(self, K: int) -> torch.Tensor:
        dev = self.A.device
        ss1 = (0.999 / self.L.to(dev)).reshape(())                  # fp32, as 0.999 / self.L
        thz = ss1 * self.alpha                                      # fp32 ss1 * alpha
        return _scalar_table(K, dev, b1=1.0, b2=1.0, b3=1.0, ss2=0.3, the=0.3, thz=thz, s1=ss1)

    def _At(self) -> torch.Tensor:
        if getattr(self, "_At_c", None) is None or self._At_c.device != self.A.device:
            self._At_c = self.A.t().contiguous()
        return self._At_c

    def _km(self, x, Z, E, L, K: int, table: Optional[torch.Tensor] = None):
        """K KM iterations from (Z, E, L) as one fused launch; T_0 = A Z + E - X.  `table`: a
        precomputed _km_table(K) (the safeguarded loop builds the 1-step table once per call)."""
        return dladmm_forward(_lib.V5_TIED, x, self.A, [self._At()] * K, Z, E, L, keep_all=True,
                              want_T=True,
                              scalar_params=self._km_table(K) if table is None else table)

    def _l2o(self, x, Z, E, L, k: int, nl: int = 1, tables: Optional[torch.Tensor] = None):
        """Learned layers k .. k+nl-1 (the V4 body, :206-227) from (Z, E, L).  `tables`: the
        module's parameter table, if the caller already assembled it for this call."""
        if tables is None:
            tables = self._tables(self.A.device)["scalar_params"]
        tab = tables[k:k + nl].contiguous()
        return dladmm_forward(_lib.V4_SCALAR, x, self.A,
                              [self.fc[j].weight.detach() for j in range(k, k + nl)], Z, E, L,
                              keep_all=True, want_T=True, scalar_params=tab)

    # --- reference methods -----------------------------------------------------------------
    def KM(self, Zk, Ek, Lk, Tk, X, **kwargs):
        """One classic KM step (:129-155) with the default constants; returns
        (Varn, Zn, En, Tn, Ln).  Tk must be A Zk + Ek - X (as everywhere in the reference)."""
        if kwargs:
            raise NotImplementedError("dladmm: KM runs with the reference defaults only")
        with torch.no_grad():
            r = self._km(X, Zk, Ek, Lk, 1)
            Varn = Lk + 1.0 * Tk
        return Varn, r.Z[0], r.E[0], r.T[1], r.L[0]

    def S(self, Zk, Ek, Lk, Tk, X, Ep, **kwargs):
        """Fixed-point residual [beta Tn ; c (En - 2 Ek + Ep)] of a KM step (:158-175)."""
        _, Zn, En, Tn, Ln = self.KM(Zk, Ek, Lk, Tk, X)
        c = sqrt(0.3 / (1 - 0.3))
        return torch.cat([1.0 * Tn, c * (En - 2 * Ek + Ep)])

    @staticmethod
    def two_norm(z, dim=0):
        return (z ** 2).sum(dim=dim).sqrt()

    def _safeguard(self, x, mu, cand_l, cand_k, s_step, Ep, out, k_out, count):
        """dladmm_safeguard_f32: |S| of the L2O candidate, mu update, per-column select."""
        L = _lib.lib()
        m, B = x.shape
        d = _lib.SafeguardDesc()
        d.abi_version = _lib.ABI_VERSION
        d.m, d.n, d.batch, d.ld = m, self.d, B, B
        d.Es, d.Ts, d.Ep, d.mu = s_step.E[0].data_ptr(), s_step.T[1].data_ptr(), Ep.data_ptr(), \
            mu.data_ptr()
        if out is None:   # mu_0 = |S(Z0, E0, L0, T0, X, E0)|
            d.El = Ep.data_ptr()
        else:
            d.Zl, d.El, d.Ll, d.Tl = (cand_l.Z[0].data_ptr(), cand_l.E[0].data_ptr(),
                                      cand_l.L[0].data_ptr(), cand_l.T[1].data_ptr())
            d.Zk, d.Ek, d.Lk, d.Tk = (cand_k.Z[0].data_ptr(), cand_k.E[0].data_ptr(),
                                      cand_k.L[0].data_ptr(), cand_k.T[1].data_ptr())
            Zo, Eo, Lo, To = out
            d.Zo, d.Eo, d.Lo = Zo[k_out].data_ptr(), Eo[k_out].data_ptr(), Lo[k_out].data_ptr()
            d.To = To[k_out + 1].data_ptr()
            d.count = count.data_ptr()
        d.beta, d.c, d.delta = 1.0, sqrt(0.3 / (1 - 0.3)), self.delta
        d.updater, d.mu_param = _UPDATERS[self.mu_k_method], self.mu_k_param
        stream = torch.cuda.current_stream(x.device).cuda_stream
        _lib.check(L.dladmm_safeguard_f32(ctypes.byref(d), ctypes.c_void_p(stream)))

    def forward(self, x, use_learned=False, use_safeguard=False, continued=False,
                K: Optional[int] = None):
        """test_syn_l1l1_scalar.py:178-316.  K defaults to the reference's
        `layers if (not continued and (use_learned or use_safeguard)) else num_iter` (:54)."""
        if K is None:
            K = self.layers if (not continued and (use_learned or use_safeguard)) else \
                self.num_iter
        if use_safeguard and not use_learned:
            raise AssertionError("safeguarding needs the learned model (:241 assert use_learned)")
        if use_learned and not continued and K > self.layers:
            raise IndexError(f"K={K} learned steps but the model has {self.layers} layers")
        nl = min(K, self.layers) if use_learned else 0
        with torch.no_grad():
            if not use_learned:
                r = self._km(x, self.Z0, self.E0, self.L0, K)
                return ([r.Z[k] for k in range(K)], [r.E[k] for k in range(K)],
                        [r.L[k] for k in range(K)], [r.T[j] for j in range(K + 1)])
            m, B = x.shape
            dev = x.device
            if use_safeguard:
                Zo = torch.empty((nl, self.d, B), device=dev)
                Eo = torch.empty((nl, m, B), device=dev)
                Lo = torch.empty((nl, m, B), device=dev)
                To = torch.empty((nl + 1, m, B), device=dev)
                count = torch.zeros(self.layers, dtype=torch.int32, device=dev)
                mu = torch.empty(B, device=dev)
                # mu_0 = |S(Z0, E0, L0, T0, X, E0)| (:190-197); T0 = A Z0 + E0 - X
                # the parameter tables of this call, assembled once (not per layer)
                km1 = self._km_table(1)
                ptab = self._tables(dev)["scalar_params"]
                s0 = self._km(x, self.Z0, self.E0, self.L0, 1, km1)
                To[0].copy_(s0.T[0])
                self._safeguard(x, mu, None, None, s0, self.E0, None, 0, None)
                Zc, Ec, Lc = self.Z0, self.E0, self.L0
                for k in range(nl):
                    cl = self._l2o(x, Zc, Ec, Lc, k, tables=ptab)          # :218-227
                    ck = self._km(x, Zc, Ec, Lc, 1, km1)                   # :215-216
                    cs = self._km(x, cl.Z[0], cl.E[0], cl.L[0], 1, km1)    # S(L2O, Ep) :244
                    self._safeguard(x, mu, cl, ck, cs, Ec, (Zo, Eo, Lo, To), k, count[k:k + 1])
                    Zc, Ec, Lc = Zo[k], Eo[k], Lo[k]
                Z, E, L, T = list(Zo), list(Eo), list(Lo), list(To)
            else:
                r = self._l2o(x, self.Z0, self.E0, self.L0, 0, nl)
                Z, E, L = list(r.Z), list(r.E), list(r.L)
                T = list(r.T)
            if continued and K > nl:   # :204-206: KM from the learned model's last iterate
                r2 = self._km(x, Z[-1], E[-1], L[-1], K - nl)
                Z += list(r2.Z)
                E += list(r2.E)
                L += list(r2.L)
                T += [r2.T[j] for j in range(1, K - nl + 1)]
            if use_safeguard:
                return Z, E, L, T, count.cpu().numpy().astype(np.float64)
            return Z, E, L, T

