"""Drop-in `DLADMMNet` modules: reference constructor, parameter names/shapes and return lists,
with the K-layer loop replaced by one fused HIP call (ops.dladmm_forward).

One class per reference variant (the reference copy-pastes a different `class DLADMMNet` into
each script):

  DLADMMNet            V1  main_lena.py:16-102            beta (m, batch_size), thetas fixed
  DLADMMNetLTheta      V2  main_syn_l1l1_ltheta.py:16-95  beta (m,1), thetas (d,1)/(m,1)
  DLADMMNetFull        V3  main_syn_l1l1_full.py:16-96    per-row beta1/2/3, ss2, thetas
  DLADMMNetScalar      V4  main_syn_l1l1_scalar.py:34-131 all (1,1); returns (Z, E, L, T)
  DLADMMNetScalarSl2 / DLADMMNetScalarZ0: V4 of main_syn_l1l1-sl2_scalar.py / _scalar_z0.py
                           (same body; name() "DLADMMNet")
  DLADMMNetScalarTied  V5  main_syn_l1l1_scalar_tied.py:34-104 one shared fc + ss1[k]
  DLADMMNetLasso       V6  main_syn_lasso_scalar.py:17-118 linear LASSO E-step

Constructor signature `(m, n, d, batch_size, A, Z0, E0, L0, layers)`, `state_dict` keys and
shapes, `name()` and the forward return arity all follow the reference, so a reference
checkpoint (e.g. DLADMMNet.pth.tar, 45 keys for V1 at layers=15) loads with
`load_state_dict(..., strict=True)` unchanged.

`forward` is differentiable: with autograd recording and parameters that require grad it runs as
the torch.autograd.Function `_DLADMMFunction`, whose backward is the HIP reverse sweep
(ops.dladmm_backward -> dladmm_bwd_f32), so `total_loss.backward(); optimizer.step()` trains the
module exactly as the reference training loops do (main_syn_l1l1_scalar.py:269-299).  Without
grad it runs the inference path (no T saved for V1-V3, nothing kept for backward).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Optional

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .ops import ForwardResult, dladmm_backward, dladmm_forward, dladmm_lena, dladmm_scale_


def _dev(t: torch.Tensor) -> torch.Tensor:
    """The reference calls .cuda() on A, Z0, E0, L0 (main_lena.py:23-26); on ROCm torch.cuda is
    the HIP device.  Without a device (CPU-only hosts) the tensors stay put so the module can
    still be built and (de)serialised; forward then raises."""
    return t.cuda() if torch.cuda.is_available() else t


class _DLADMMBase(nn.Module):
    VARIANT = 0
    RETURNS_T = False
    WSCALE = 1.0     # fc init scale: main_lena.py:49 (1.0) / main_syn_l1l1_scalar.py:72 (0.4)
    NAME = "DLADMMNet"

    def __init__(self, m, n, d, batch_size, A, Z0, E0, L0, layers, *, batch_shard=None):
        """The reference constructor (main_lena.py:17-49), plus the keyword `batch_shard=(rank,
        world)`: build rank `rank`'s share of a data-parallel run directly -- Z0 / E0 / L0 given
        with batch_size columns are sliced to the rank's span (on their own device, before the
        move to the GPU; already-sliced ones are taken as they are) and V1's per-sample betas
        are registered at (m, c1 - c0) from the start, so no rank ever holds the global
        2 K m batch_size betas (main_lena.py:35-36).  Same parameters, names and initial values
        as the replicated module followed by shard_batch_(rank, world)."""
        super().__init__()
        self.m = m
        self.n = n
        self.d = d
        self.batch_size = batch_size
        self.layers = layers
        self.batch_shard = None   # (c0, c1, batch_size) of a data-parallel shard
        cols = None
        if batch_shard is not None:
            from .dist import shard_columns
            rank, world = (int(x) for x in batch_shard)
            cols = shard_columns(batch_size, rank, world)
            Z0, E0, L0 = (_shard_cols(t, batch_size, cols, nm)
                          for t, nm in ((Z0, "Z0"), (E0, "E0"), (L0, "L0")))
        self.A = _dev(A)
        self.Z0 = _dev(Z0)
        self.E0 = _dev(E0)
        self.L0 = _dev(L0)
        # columns of the per-sample parameters this module holds (V1's betas)
        self._pcols = batch_size if cols is None else cols[1] - cols[0]
        self._register_params()
        self._init_fc()
        if cols is not None:
            self.batch_shard = (cols[0], cols[1], batch_size)
            self.world = (rank, world)
        # the reference follows construction with model.cuda() (main_lena.py:191); do it here
        self.to(self.A.device)

    # --- construction -----------------------------------------------------------------
    def _plist(self, name, shape, value):
        pl = nn.ParameterList()
        for _ in range(self.layers):
            pl.append(nn.Parameter(value * torch.ones(*shape, dtype=torch.float32)))
        setattr(self, name, pl)

    def _register_params(self):  # pragma: no cover - per variant
        raise NotImplementedError

    def _init_fc(self):
        # main_lena.py:45-49 / main_syn_l1l1_scalar.py:67-72: every Linear's weight is replaced by
        # s * (A^T + 1e-3 * N(0, 1)), on A's device
        for mod in self.modules():
            if isinstance(mod, nn.Linear):
                w = self.A.t() + (1e-3) * torch.randn_like(self.A.t())
                if self.WSCALE != 1.0:
                    w = w * self.WSCALE
                # A.t() + noise inherits A.t()'s column-major strides; store it row-major (same
                # values, same state_dict) so the weight packer reads rows
                mod.weight = nn.Parameter(w.contiguous())

    def name(self):
        return self.NAME

    # --- data parallelism ----------------------------------------------
    def _elem_param_lists(self) -> list:
        """The ParameterLists whose entries are per-sample (m, batch_size): V1's beta1 / beta2
        (main_lena.py:35-36).  Other variants: none (their parameters are replicated)."""
        return []

    def shard_batch_(self, rank: int, world: int):
        """Make this module rank `rank`'s share of a data-parallel run over `world` ranks (in
        place): it keeps only its contiguous column span c0:c1 = dist.shard_columns(batch_size,
        rank, world) of everything that is per sample -- Z0, E0, L0 and V1's per-sample betas
        (main_lena.py:35-36), which become (m, c1 - c0) Parameters holding their current values'
        columns (rank-local: dist.rank_local_params finds them from the module).  Then:
          * forward / training_loss take the rank's (m, c1 - c0) shard of X; training_loss's
            mean runs over the global batch_size by default, so the ranks' gradients SUM to the
            whole batch's;
          * dist.allreduce_grads all-reduces only the replicated parameters (W_k, scalar and
            per-row ones): a per-sample beta's gradient is rank-local;
          * load_state_dict slices a global checkpoint's (m, batch_size) betas to the span, and
            dist.gather_state_dict assembles the reference layout again for saving.
        Per rank, V1's betas then cost 2 K m (B / world) floats instead of 2 K m B (the global
        betas exist until this call; the constructor's batch_shard= never makes them).  Returns
        self."""
        from .dist import shard_columns
        if self.batch_shard is not None:
            raise RuntimeError("dladmm: the module is already a batch shard")
        B = self.Z0.shape[1]
        for pl in self._elem_param_lists():
            if any(q.shape[1] != B for q in pl):
                raise ValueError("dladmm: per-sample parameters and Z0 disagree on the batch")
        c0, c1 = shard_columns(B, rank, world)
        self.Z0 = self.Z0[:, c0:c1].contiguous()
        self.E0 = self.E0[:, c0:c1].contiguous()
        self.L0 = self.L0[:, c0:c1].contiguous()
        for pl in self._elem_param_lists():
            for i in range(len(pl)):
                pl[i] = nn.Parameter(pl[i].detach()[:, c0:c1].contiguous(),
                                     requires_grad=pl[i].requires_grad)
        self._pcols = c1 - c0
        self.batch_shard = (c0, c1, B)
        self.world = (rank, world)
        return self

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """nn.Module.load_state_dict; on a batch shard (shard_batch_) a per-sample beta given in
        the global (m, batch_size) layout of a reference checkpoint is sliced to the shard's
        columns first."""
        if self.batch_shard is not None:
            c0, c1, B = self.batch_shard
            names = {f"{nm}.{k}" for nm in self._elem_names() for k in range(self.layers)}
            sd = OrderedDict(state_dict)
            for key in names & set(sd):
                v = sd[key]
                if torch.is_tensor(v) and v.dim() == 2 and v.shape[1] == B and c1 - c0 != B:
                    sd[key] = v[:, c0:c1]
            state_dict = sd
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    def _elem_names(self) -> list:
        return [nm for nm, mod in self.named_children() if any(mod is pl for pl in
                                                               self._elem_param_lists())]

    # --- fused forward ----------------------------------------------------------------
    def _weights(self) -> List[torch.Tensor]:
        return [self.fc[k].weight for k in range(self.layers)]

    def _table_spec(self) -> dict:  # pragma: no cover - per variant
        """{"scalar" | "row": {slot: source}}: which parameter feeds which slot of the C ABI's
        per-layer table.  A source is a ParameterList (one entry per layer), a 0-dim tensor
        (every layer) or a float constant."""
        raise NotImplementedError

    def _elem_betas(self, cols=None) -> dict:
        """V1's per-sample betas (passed to the C ABI by pointer, read live); others: none."""
        return {}

    def _tables(self, dev, cols=None) -> dict:
        """Per-layer parameter tables for the C ABI, assembled from the live parameters on every
        call (one cat + one index_copy, _assemble_table).  Nothing is cached across calls:
        an optimizer step, load_state_dict, or an in-place edit through p.data (which does not
        bump the version counter) all take effect on the next call."""
        out = {}
        for kind, spec in self._table_spec().items():
            R = 1 if kind == "scalar" else max(self.m, self.d)
            rows = {nm: (1 if kind == "scalar" else (self.d if nm == "thz" else self.m))
                    for nm in spec}
            out[f"{kind}_params"] = _assemble_table(self.layers, R, dev, spec, rows)
        out.update(self._elem_betas(cols))
        return out

    def _needs_grad(self) -> bool:
        return torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())

    # GEMM precision of forward / run: "f32" (fp32 MFMA: every GEMM an exact fp32 fma chain),
    # "f32_split" (the same fp32 GEMMs on the f16 matrix cores: operands split exactly into
    # scaled hi + lo f16 halves, hi*hi + hi*lo + lo*hi accumulated in fp32 -- the error of an fp32
    # GEMM, ~3x the throughput; V1 and V4-V6 at the fused shapes, V2 / V3 run f32) or "bf16"
    # (BASELINE config 5:
    # bf16 MFMA operands, fp32 accumulation and fp32 elementwise state).  Training runs "f32" or
    # "f32_split": the split-f16 forward saves the product A Z_k its updates consumed, and the
    # (fp32) backward differentiates that forward; "bf16" is inference-only.
    precision = "f32"

    def run(self, x: torch.Tensor, keep_all: bool = True, loss_kind: int = 0,
            kernel_events=None, want_col_loss: bool = False):
        """Fused forward returning the raw ops.ForwardResult (stacked [K, rows, B] outputs).
        Not differentiable (it is the inference path; `forward` is the differentiable one)."""
        with torch.no_grad():
            dev = self.A.device
            return dladmm_forward(
                self.VARIANT, x, self.A, [w.detach() for w in self._weights()],
                self.Z0, self.E0, self.L0, keep_all=keep_all, want_T=self.RETURNS_T,
                loss_kind=loss_kind, kernel_events=kernel_events, want_col_loss=want_col_loss,
                precision=self.precision, **self._tables(dev))

    def _forward_layers(self, x, nl: int):
        """Run the first `nl` layers; lists Z, E, L (nl entries) and T (nl + 1), differentiable
        when autograd records and parameters require grad."""
        if self._needs_grad():
            if x.requires_grad:
                raise RuntimeError("dladmm: gradients w.r.t. the input X are not supported (the "
                                   "reference trains the parameters only)")
            if self.precision not in ("f32", "f32_split"):
                raise RuntimeError(f"dladmm: precision {self.precision!r} is inference-only "
                                   "(training runs f32 or f32_split)")
            outs = _DLADMMFunction.apply(self, x, nl, *self.parameters())
            return (list(outs[:nl]), list(outs[nl:2 * nl]), list(outs[2 * nl:3 * nl]),
                    list(outs[3 * nl:]))
        with torch.no_grad():
            tables = _slice_tables(self._tables(self.A.device), nl)
            r = dladmm_forward(self.VARIANT, x, self.A, [w.detach() for w in self._weights()[:nl]],
                               self.Z0, self.E0, self.L0, keep_all=True, want_T=self.RETURNS_T,
                               precision=self.precision, **tables)
        T = [r.T[j] for j in range(nl + 1)] if r.T is not None else None
        return ([r.Z[k] for k in range(nl)], [r.E[k] for k in range(nl)],
                [r.L[k] for k in range(nl)], T)

    def forward(self, x):
        Z, E, L, T = self._forward_layers(x, self.layers)
        if self.RETURNS_T:
            return Z, E, L, T
        return Z, E, L

    def layer_objectives(self, x, alpha: float, kind: str = "l1l1", kernel_events=None,
                         want_col_loss: bool = False):
        """Forward + the per-layer objective of the reference training loop, fused in-kernel:
        l1l1  alpha*sum(|Z_k|,0).mean() + sum(|X - A Z_k|,0).mean()   main_syn_l1l1_scalar.py:290-294
        lasso alpha*sum(|Z_k|,0).mean() + 0.5*sum((X-A Z_k)^2,0).mean() main_syn_lasso_scalar.py:276-281
        Returns (ForwardResult, fp64 tensor [K]); want_col_loss also fills ForwardResult.col_loss
        [K, 2, B] with the per-column (sum|Z_k|, fit) terms."""
        lk = {"l1l1": _lib.LOSS_L1L1, "lasso": _lib.LOSS_LASSO}[kind]
        r = self.run(x, loss_kind=lk, kernel_events=kernel_events, want_col_loss=want_col_loss)
        obj = (alpha * r.loss_sums[:, 0] + r.loss_sums[:, 1]) / x.shape[1]
        return r, obj

    def training_loss(self, x, alpha: float, coeffs=None, kind: str = "l1l1",
                      batch: Optional[int] = None, cols=None, lx_sign: float = 1.0,
                      save_cotangents: bool = True):
        """The reference training objective as one fused, differentiable op:
            total = sum_k coeffs[k] * (alpha * sum(|Z_k|,0).mean() + sum(|X - A Z_k|,0).mean())
        (main_syn_l1l1_scalar.py:283-296; kind='lasso': 0.5*sum((X - A Z_k)^2,0), lasso
        :270-283; kind='lena': main_lena.py:221-228,
            l_k = alpha*mean|Z_k| + mean|E_k| + mean(dual_gap(A^T L_k, alpha))
                  + mean(dual_gap(L_k, 1)) + mean(L_k * X),
        dual_gap(x, c) = softplus(x - c) + softplus(-x - c) (:145-147), the means over all
        elements; m <= 256, n <= 512; lx_sign=-1 gives main_syn_l1l1-dgap_ltheta.py:201-207's
        `- mean(L_k * X)`, whose loop also zeroes the layers below loss_start_layer = layers - 1:
        coeffs [0, ..., 0, 1]).  coeffs default: all 1; the reference uses decay 0.6**epoch
        for k < K-1.
        kind='lena' keeps, between forward and backward, the E_k / L_k cotangents the training
        forward forms in the same pass as the sums (2 K m B fp32 beside the saved layers, outside
        save_for_backward: saved-tensor hooks do not see them); save_cotangents=False forms them
        in the backward instead (one more pass over the K products A^T L_k).
        Returns (total, per-layer losses [K]); call total.backward() as the reference does.
        Mathematically the same gradients as building the loss from forward()'s outputs with
        torch ops, without the K products A Z_k.

        Data-parallel shards: `cols` = (c0, c1) runs the columns c0..c1-1 of the model's batch
        (x is that shard, (m, c1 - c0); Z0/E0/L0 and V1's per-sample betas are sliced to it) and
        `batch` = the column count of the mean (default x.shape[1]; pass the global batch).
        Each rank's gradient is then its shard's share of the global objective, and
        dist.allreduce_grads (SUM) gives the full-batch gradient."""
        K = self.layers
        coeffs = [1.0] * K if coeffs is None else [float(c) for c in coeffs]
        if len(coeffs) != K:
            raise ValueError(f"dladmm: coeffs must have {K} entries")
        if kind not in ("l1l1", "lasso", "lena"):
            raise ValueError(f"dladmm: unknown loss kind {kind!r}")
        if cols is not None and self.batch_shard is not None:
            raise ValueError("dladmm: cols= slices a replicated model; a batch shard "
                             "(shard_batch_) takes its own columns' x directly")
        if batch is None and self.batch_shard is not None:
            batch = self.batch_shard[2]   # the mean over the global batch
        if cols is not None:
            cols = (int(cols[0]), int(cols[1]))
            # an empty shard (c0 == c1: dist.shard_columns when the batch has fewer columns
            # than ranks) is valid: it contributes zero, and its rank still joins the collectives
            if not (0 <= cols[0] <= cols[1] <= self.Z0.shape[1]) or \
                    x.shape[1] != cols[1] - cols[0]:
                raise ValueError(f"dladmm: cols {cols} do not match x {tuple(x.shape)} and the "
                                 f"model's batch of {self.Z0.shape[1]} columns")
        denom = float(batch if batch is not None else x.shape[1])
        if kind == "lena":
            lx_sign = float(lx_sign)
            if lx_sign not in (1.0, -1.0):
                raise ValueError(f"dladmm: lx_sign must be +1 or -1 (got {lx_sign})")
            if self._needs_grad():
                if x.requires_grad:
                    raise RuntimeError("dladmm: gradients w.r.t. the input X are not supported")
                return _DLADMMLenaLossFunction.apply(self, x, coeffs, float(alpha), denom, cols,
                                                     lx_sign, bool(save_cotangents),
                                                     *self.parameters())
            # evaluation: the module's own precision, nothing saved, the sums only (mode 0)
            with torch.no_grad():
                r = self._run_shard(x, cols, loss_kind=_lib.LOSS_L1L1, want_T=False)
                sums = dladmm_lena(x, self.A, r.E, r.L, float(alpha), denom, lx_sign=lx_sign)
                per_layer = _lena_per_layer(r.loss_sums, sums, float(alpha), self.A.shape,
                                            denom, lx_sign)
                c = _coef_tensor(coeffs, per_layer.device)
                return (c * per_layer).sum().to(torch.float32), per_layer.to(torch.float32)
        if self._needs_grad():
            if x.requires_grad:
                raise RuntimeError("dladmm: gradients w.r.t. the input X are not supported")
            return _DLADMMLossFunction.apply(self, x, coeffs, float(alpha), kind, denom, cols,
                                             *self.parameters())
        lk = {"l1l1": _lib.LOSS_L1L1, "lasso": _lib.LOSS_LASSO}[kind]
        with torch.no_grad():
            r = self._run_shard(x, cols, loss_kind=lk, want_T=self.RETURNS_T)
        per_layer = (alpha * r.loss_sums[:, 0] + r.loss_sums[:, 1]) / denom
        c = _coef_tensor(coeffs, per_layer.device)
        return (c * per_layer).sum().to(torch.float32), per_layer.to(torch.float32)

    def _init_state(self, cols=None):
        """(Z0, E0, L0) of the whole model batch or of the column shard cols = (c0, c1)."""
        if cols is None:
            return self.Z0, self.E0, self.L0
        c0, c1 = cols
        return self.Z0[:, c0:c1], self.E0[:, c0:c1], self.L0[:, c0:c1]

    def _run_shard(self, x, cols, **kw):
        """Forward of every layer on the column shard `cols` (None: the whole batch), at the
        module's precision unless `precision=` is given."""
        dev = self.A.device
        Z0, E0, L0 = self._init_state(cols)
        W = [w.detach() for w in self._weights()]
        kw.setdefault("precision", self.precision)
        return dladmm_forward(self.VARIANT, x, self.A, W, Z0, E0, L0, keep_all=True,
                              **kw, **self._tables(dev, cols))

    # --- backward: map the C ABI's gradient tables onto the reference parameters ------------
    # GRAD_SLOTS: ParameterList name -> (kind, slots summed).  kind 'scalar' reads g_scalar,
    # 'row' reads g_row (theta_z rows = d, else m), 'elem1'/'elem2' the V1 per-sample betas.
    GRAD_SLOTS: dict = {}
    # which update steps of a layer read each parameter: z = Z-step (Var, shrink of Z), e = E-step,
    # l = L-step.  V1/V2 use beta1 for Var and L (main_lena.py:85,89): "zl".
    PARAM_STEPS = {"beta1": "z", "beta2": "e", "beta3": "l", "ss2": "e", "ss2_1": "e",
                   "ss2_2": "e", "ss1": "z", "active_para": "z", "active_para1": "e"}

    def _fc_key(self, k: int) -> str:
        """state_dict key of the weight layer k uses."""
        return "fc.weight" if self._shared_weight() else f"fc.{k}.weight"

    def _param_grads(self, res, nl: int, reach: Optional[dict] = None, cols=None) -> dict:
        """Gradients by state_dict key from a BackwardResult of the first `nl` layers.  As in the
        reference's autograd, a parameter no cotangent can reach gets None, not a zero tensor:
        layers >= nl were not run, and `reach` (_reachable) marks the layer steps the loss
        depends on.  cols = (c0, c1): the forward ran on that column shard of a (m, batch_size)
        V1 beta, whose gradient is zero outside it."""
        out = {}
        rz = reach["z"] if reach else [True] * nl
        # one fp64 -> fp32 conversion per table; a single-slot gradient is then a view of it
        # (per-parameter sum / cast ops were ~180 tiny launches per training step)
        kinds = {kind for kind, _ in self.GRAD_SLOTS.values()}
        gs32 = res.g_scalar.to(torch.float32) if "scalar" in kinds else None
        gr32 = res.g_row.to(torch.float32) if "row" in kinds else None
        for name, (kind, slots) in self.GRAD_SLOTS.items():
            steps = self.PARAM_STEPS[name]
            for k in range(nl):
                if reach is not None and not any(reach[s][k] for s in steps):
                    continue
                key = f"{name}.{k}"
                if kind == "scalar":
                    g = (gs32[k, slots[0]] if len(slots) == 1 else
                         sum(res.g_scalar[k, s] for s in slots).to(torch.float32)).reshape(1, 1)
                elif kind == "row":
                    rows = self.d if slots[0] == _lib.P_THETA_Z else self.m
                    g = (gr32[k, slots[0], :rows] if len(slots) == 1 else
                         sum(res.g_row[k, s, :rows] for s in slots).to(torch.float32))
                    g = g.reshape(rows, 1)
                else:
                    g = (res.g_beta1 if kind == "elem1" else res.g_beta2)[k].to(torch.float32)
                    if cols is not None:
                        full = torch.zeros((self.m, self.batch_size), dtype=torch.float32,
                                           device=g.device)
                        full[:, cols[0]:cols[1]] = g
                        g = full
                out[key] = g
        if self._shared_weight():
            if any(rz[:nl]):
                out[self._fc_key(0)] = res.gW[0]
        else:
            for k in range(nl):
                if not rz[k]:
                    continue
                key = self._fc_key(k)
                out[key] = res.gW[k] if key not in out else out[key] + res.gW[k]
        return out

    def _shared_weight(self) -> bool:
        return isinstance(self.fc, nn.Linear)


def _shard_cols(t: torch.Tensor, batch: int, cols, name: str) -> torch.Tensor:
    """Rank's columns c0:c1 of a (rows, batch) initial-state tensor; a tensor that already has
    c1 - c0 columns is the caller's shard and is taken as it is."""
    c0, c1 = cols
    if t.dim() == 2 and t.shape[1] == batch and c1 - c0 != batch:
        return t[:, c0:c1].contiguous()
    if t.dim() == 2 and t.shape[1] == c1 - c0:
        return t
    raise ValueError(f"dladmm: {name} of shape {tuple(t.shape)} is neither the global batch "
                     f"({batch} columns) nor the shard's {c1 - c0}")


def _slice_tables(tables: dict, nl: int) -> dict:
    """Per-layer parameter tables of the first nl layers."""
    return {k: (v[:nl] if v is not None else None) for k, v in tables.items()}


def _train_precision(mod) -> str:
    """Forward precision of a differentiable call: the module's "f32_split" (which saves its own
    A Z_k for the backward), else "f32"."""
    if mod.precision not in ("f32", "f32_split"):
        raise RuntimeError(f"dladmm: precision {mod.precision!r} is inference-only "
                           "(training runs f32 or f32_split)")
    return mod.precision


class _DLADMMFunction(torch.autograd.Function):
    """The K-layer forward as one differentiable op: forward = dladmm_fwd_f32 with every layer
    (and T) saved, backward = dladmm_bwd_f32 (the HIP reverse sweep).

    Inputs: the module, X, and the module's parameters in `parameters()` order.  Outputs: the
    4K+1 per-layer tensors Z_0..Z_{K-1}, E_0.., L_0.., T_0..T_K as SEPARATE outputs (views of one
    stacked buffer each), so autograd hands back one cotangent per layer -- or None for a layer
    the loss never reads -- instead of accumulating K zero-filled stacks."""

    @staticmethod
    def forward(ctx, mod, x, nl, *params):
        dev = mod.A.device
        tables = _slice_tables(mod._tables(dev), nl)
        W = [w.detach() for w in mod._weights()[:nl]]
        r = dladmm_forward(mod.VARIANT, x, mod.A, W, mod.Z0, mod.E0, mod.L0, keep_all=True,
                           want_T=True, want_P=True, precision=_train_precision(mod), **tables)
        ctx.mod = mod
        ctx.nl = nl
        ctx.tables = tables
        ctx.W = W
        ctx.fpath = r.path  # the forward's kernel path (4: split-f16, see dladmm_backward)
        ctx.fflags = r.flags  # its plan options: the backward runs on an autograd thread
        ctx.save_for_backward(x, r.Z, r.E, r.L, r.T, r.P)
        ctx.set_materialize_grads(False)
        K = nl
        outs = tuple(r.Z[k] for k in range(K)) + tuple(r.E[k] for k in range(K)) + \
            tuple(r.L[k] for k in range(K)) + tuple(r.T[j] for j in range(K + 1))
        if not mod.RETURNS_T:
            ctx.mark_non_differentiable(*outs[3 * K:])
        return outs

    @staticmethod
    def backward(ctx, *g):
        x, Z, E, L, T, P = ctx.saved_tensors
        mod = ctx.mod
        K = ctx.nl
        saved = ForwardResult(Z, E, L, T, None, P=P, path=ctx.fpath, flags=ctx.fflags)
        res = dladmm_backward(mod.VARIANT, x, mod.A, ctx.W, mod.Z0, mod.E0, mod.L0, saved,
                              g[:K], g[K:2 * K], g[2 * K:3 * K],
                              g[3 * K:] if mod.RETURNS_T else None,
                              tied=mod._shared_weight(), **ctx.tables)
        grads = mod._param_grads(res, K, _reachable(K, g, mod.RETURNS_T))
        names = [n for n, _ in mod.named_parameters()]
        return (None, None, None) + tuple(grads.get(n) for n in names)


_COEF: "OrderedDict" = OrderedDict()


def _coef_tensor(coeffs, dev) -> torch.Tensor:
    """The layer coefficients as a device fp64 vector, cached per (device, values): a training
    step then makes no host-to-device copy once warm, so it can be captured into a HIP graph
    (tests/test_gpu_graph.py).  A handful of entries (the reference decays them per epoch)."""
    key = (str(dev), tuple(coeffs))
    c = _COEF.pop(key, None)
    if c is None:
        c = torch.as_tensor(list(coeffs), dtype=torch.float64, device=dev)
    _COEF[key] = c
    while len(_COEF) > 16:
        _COEF.popitem(last=False)
    return c


class _DLADMMLossFunction(torch.autograd.Function):
    """The reference training objective fused into the op (SURVEY.md section 8 rows a11 + f1):
        total = sum_k coeffs[k] * (alpha * sum(|Z_k|, 0).mean() + sum(|X - A Z_k|, 0).mean())
    (main_syn_l1l1_scalar.py:283-296; LASSO main_syn_lasso_scalar.py:270-283 with
    0.5*sum((X - A Z_k)^2, 0)), computed from the forward kernel's per-layer sums and
    differentiated inside the backward kernels -- the K products A Z_k of the reference loss
    never run.  Outputs: total (0-dim, differentiable) and the per-layer losses [K]
    (non-differentiable, for logging as the reference prints loss[k])."""

    @staticmethod
    def forward(ctx, mod, x, coeffs, alpha, kind, denom, cols, *params):
        dev = mod.A.device
        tables = mod._tables(dev, cols)
        W = [w.detach() for w in mod._weights()]
        Z0, E0, L0 = mod._init_state(cols)
        lk = {"l1l1": _lib.LOSS_L1L1, "lasso": _lib.LOSS_LASSO}[kind]
        r = dladmm_forward(mod.VARIANT, x, mod.A, W, Z0, E0, L0, keep_all=True, want_T=True,
                           loss_kind=lk, want_P=True, precision=_train_precision(mod), **tables)
        per_layer = (alpha * r.loss_sums[:, 0] + r.loss_sums[:, 1]) / denom  # fp64 [K]
        c = _coef_tensor(coeffs, dev)
        total = (c * per_layer).sum().to(torch.float32)
        ctx.mod, ctx.tables, ctx.W, ctx.lk, ctx.cols = mod, tables, W, lk, cols
        # (cz_k, cf_k) per unit upstream gradient
        ctx.base = torch.stack([c * alpha / denom, c / denom], 1).to(torch.float32)
        ctx.fpath = r.path  # the forward's kernel path (4: split-f16, see dladmm_backward)
        ctx.fflags = r.flags  # its plan options: the backward runs on an autograd thread
        ctx.save_for_backward(x, r.Z, r.E, r.L, r.T, r.P)
        per_layer = per_layer.to(torch.float32)
        ctx.mark_non_differentiable(per_layer)
        return total, per_layer

    @staticmethod
    def backward(ctx, g_total, g_layers):
        x, Z, E, L, T, P = ctx.saved_tensors
        mod = ctx.mod
        K = mod.layers
        coef = (ctx.base * g_total).contiguous()  # device-side scale, no host sync
        Z0, E0, L0 = mod._init_state(ctx.cols)
        res = dladmm_backward(mod.VARIANT, x, mod.A, ctx.W, Z0, E0, L0,
                              ForwardResult(Z, E, L, T, None, P=P, path=ctx.fpath,
                                            flags=ctx.fflags),
                              loss_kind=ctx.lk,
                              loss_coef=coef,
                              tied=mod._shared_weight(), **ctx.tables)
        # the objective reads Z_0..Z_{K-1} only: the last layer's E/L steps feed nothing
        reach = {"z": [True] * K, "e": [k < K - 1 for k in range(K)],
                 "l": [k < K - 1 for k in range(K)]}
        grads = mod._param_grads(res, K, reach, ctx.cols)
        names = [n for n, _ in mod.named_parameters()]
        return (None,) * 7 + tuple(grads.get(n) for n in names)


class _DLADMMLenaLossFunction(torch.autograd.Function):
    """main_lena.py's training objective (:221-228; dual_gap :145-147) as one differentiable op:
        total = sum_k coeffs[k] * (alpha mean|Z_k| + mean|E_k| + mean dual_gap(A^T L_k, alpha)
                                   + mean dual_gap(L_k, 1) + mean(L_k X)).
    Forward: the fused K-layer kernel (its sum|Z_k| partials) + dladmm_lena_f32 -- mode 0 (the
    other four sums; A^T L_k is formed and reduced in registers, never stored) when no gradient
    is wanted, else mode 2: the same sums and, in the same pass, the E_k / L_k cotangents of
    sum_k c_k l_k (the product A S_k of the dual_gap term included).  Backward: those cotangents
    times the upstream gradient (dladmm_scale_f32: no pass at all for total.backward()'s 1) into
    dladmm_bwd_f32, with alpha mean|Z_k| as its fused |Z| term -- the reverse sweep where the
    shape has it.  The reference instead forms the K products
    A^T L_k and a dozen elementwise passes over them with torch ops, and autograd as many more.
    Outputs: total (0-dim) and the per-layer losses [K] (non-differentiable)."""

    @staticmethod
    def forward(ctx, mod, x, coeffs, alpha, denom, cols, lx_sign, save_cot, *params):
        dev = mod.A.device
        tables = mod._tables(dev, cols)
        W = [w.detach() for w in mod._weights()]
        Z0, E0, L0 = mod._init_state(cols)
        r = dladmm_forward(mod.VARIANT, x, mod.A, W, Z0, E0, L0, keep_all=True, want_T=True,
                           loss_kind=_lib.LOSS_L1L1, want_P=True, precision=_train_precision(mod),
                           **tables)
        c = _coef_tensor(coeffs, dev)
        c32 = c.to(torch.float32)
        ctx.grad = any(ctx.needs_input_grad[8:])
        if ctx.grad and save_cot:
            # a training forward: the sums and the cotangents of sum_k c_k l_k in one pass
            # (mode 2); the backward scales the cotangents by its upstream gradient
            sums, gE, gL = dladmm_lena(x, mod.A, r.E, r.L, alpha, denom, coef=c32,
                                       lx_sign=lx_sign)
        else:
            # the sums only (mode 0); a backward forms the cotangents itself (mode 1)
            sums = dladmm_lena(x, mod.A, r.E, r.L, alpha, denom, lx_sign=lx_sign)
            gE = gL = None
        per_layer = _lena_per_layer(r.loss_sums, sums, alpha, mod.A.shape, denom, lx_sign)
        total = (c * per_layer).sum().to(torch.float32)
        ctx.mod, ctx.tables, ctx.W, ctx.cols = mod, tables, W, cols
        ctx.alpha, ctx.denom, ctx.lx_sign = alpha, denom, lx_sign
        ctx.c = c32
        ctx.gEL = (gE, gL)
        ctx.fpath = r.path  # the forward's kernel path (4: split-f16, see dladmm_backward)
        ctx.fflags = r.flags  # its plan options: the backward runs on an autograd thread
        ctx.save_for_backward(x, r.Z, r.E, r.L, r.T, r.P)
        per_layer = per_layer.to(torch.float32)
        ctx.mark_non_differentiable(per_layer)
        return total, per_layer

    @staticmethod
    def backward(ctx, g_total, g_layers):
        x, Z, E, L, T, P = ctx.saved_tensors
        mod = ctx.mod
        K = mod.layers
        m, n = mod.A.shape
        ck = (ctx.c * g_total).contiguous()                     # device-side, no host sync
        gE, gL = ctx.gEL if ctx.gEL is not None else (None, None)
        ctx.gEL = None
        if gE is None:
            # a second backward through a retained graph: the first scaled the forward's
            # cotangents in place, so form them again (mode 1)
            gE, gL = dladmm_lena(x, mod.A, E, L, ctx.alpha, ctx.denom, coef=ctx.c, sums=False,
                                 lx_sign=ctx.lx_sign)
        g1 = g_total.to(torch.float32).reshape(1).contiguous()
        dladmm_scale_(gE, g1)   # a launch that returns at once for total.backward()'s 1
        dladmm_scale_(gL, g1)
        # alpha mean|Z_k| as the backward's fused |Z| term; no fit term
        coef = torch.stack([ck * (ctx.alpha / (n * ctx.denom)), torch.zeros_like(ck)],
                           1).contiguous()
        Z0, E0, L0 = mod._init_state(ctx.cols)
        res = dladmm_backward(mod.VARIANT, x, mod.A, ctx.W, Z0, E0, L0,
                              ForwardResult(Z, E, L, T, None, P=P, path=ctx.fpath,
                                            flags=ctx.fflags),
                              gE=[gE[k] for k in range(K)], gL=[gL[k] for k in range(K)],
                              loss_kind=_lib.LOSS_L1L1, loss_coef=coef,
                              tied=mod._shared_weight(), **ctx.tables)
        reach = {"z": [True] * K, "e": [True] * K, "l": [True] * K}
        grads = mod._param_grads(res, K, reach, ctx.cols)
        names = [n_ for n_, _ in mod.named_parameters()]
        return (None,) * 8 + tuple(grads.get(n_) for n_ in names)


def _lena_per_layer(loss_sums, sums, alpha, shape, denom, lx_sign):
    """fp64 [K] per-layer values of main_lena.py:221-228 from the forward's sum|Z_k| (loss_sums
    [:, 0]) and dladmm_lena's four sums (|E_k|, dual_gap(A^T L_k, alpha), dual_gap(L_k, 1),
    L_k X); lx_sign -1: main_syn_l1l1-dgap_ltheta.py:205."""
    m, n = shape
    return (alpha * loss_sums[:, 0] / n + sums[:, 1] / n +
            (sums[:, 0] + sums[:, 2] + lx_sign * sums[:, 3]) / m) / denom


def _reachable(K: int, g, has_t: bool) -> dict:
    """Which layer steps of a K-layer forward the cotangents g (Z_0..Z_{K-1}, E.., L..,
    T_0..T_K; None = not read) depend on, as reference autograd sees the graph:
      E-step k: E_k feeds T_{k+1}, L_k and everything after layer k
      L-step k: L_k feeds layer k+1 (Var, E-step, L) but not T_{k+1}
      Z-step k: Z_k feeds E_k (through A Z_k) and Z_{k+1}
    Returns {"z" | "e" | "l": [bool] * K}."""
    def suffix(seq, n):
        out, acc = [False] * (n + 1), False
        for i in range(n - 1, -1, -1):
            acc = acc or (seq is not None and seq[i] is not None)
            out[i] = acc
        return out
    gZ, gE, gL = g[:K], g[K:2 * K], g[2 * K:3 * K]
    gT = g[3 * K:] if has_t else None
    sZ, sE, sL, sT = suffix(gZ, K), suffix(gE, K), suffix(gL, K), suffix(gT, K + 1)
    sT = sT + [False]
    re = [sE[k] or sL[k] or sT[k + 1] or sZ[k + 1] for k in range(K)]
    rl = [sL[k] or sZ[k + 1] or sE[k + 1] or sT[k + 2] for k in range(K)]
    rz = [sZ[k] or re[k] for k in range(K)]
    return {"z": rz, "e": re, "l": rl}


_SLOTS = {"b1": _lib.P_BETA1, "b2": _lib.P_BETA2, "b3": _lib.P_BETA3, "ss2": _lib.P_SS2,
          "ss2b": _lib.P_SS2B, "the": _lib.P_THETA_E, "thz": _lib.P_THETA_Z, "s1": _lib.P_S1}
_TABLE_IDX = {}


def _assemble_table(K: int, R: int, dev, spec: dict, rows: dict) -> torch.Tensor:
    """(K, 8) fp32 table (R = 1) or (K, 8, R) per-row table of the C ABI from the live
    parameter values: ONE torch.cat of every source plus ONE index_copy into a base holding the
    constant slots (missing slots 0).  The scatter index depends only on the layout and is built
    once per (device, layout)."""
    tensors, layout = [], []
    consts = []
    for nm, src in spec.items():
        if isinstance(src, (int, float)):
            consts.append((nm, float(src)))
            continue
        seq = [src] * K if torch.is_tensor(src) else list(src)
        if len(seq) < K:
            raise ValueError(f"dladmm: {len(seq)} entries for parameter slot {nm}, need {K}")
        layout.append((nm, rows[nm]))
        tensors += [t.detach().reshape(-1) for t in seq[:K]]
    key = (str(dev), K, R, tuple(layout), tuple(consts))
    ent = _TABLE_IDX.get(key)
    if ent is None:
        idx = []
        for nm, nr in layout:
            for k in range(K):
                base = (k * _lib.NSCALAR + _SLOTS[nm]) * R
                idx.extend(range(base, base + nr))
        base_t = torch.zeros(K * _lib.NSCALAR * R, dtype=torch.float32)
        for nm, v in consts:
            for k in range(K):
                o = (k * _lib.NSCALAR + _SLOTS[nm]) * R
                base_t[o:o + R] = v
        ent = (torch.tensor(idx, dtype=torch.int64).to(dev), base_t.to(dev))
        _TABLE_IDX[key] = ent
    idx, base_t = ent
    out = base_t.clone()
    if tensors:
        flat = torch.cat(tensors).to(device=dev, dtype=torch.float32)
        if flat.numel() != idx.numel():
            raise ValueError("dladmm: parameter shapes do not match the table layout")
        out.index_copy_(0, idx, flat)
    return out.view(K, _lib.NSCALAR) if R == 1 else out.view(K, _lib.NSCALAR, R)


def _scalar_table(K, dev, **cols) -> torch.Tensor:
    """(K, 8) fp32 table of per-layer scalars from floats / 0-dim tensors (KM constants)."""
    t = torch.zeros((K, _lib.NSCALAR), dtype=torch.float32, device=dev)
    for k, v in cols.items():
        t[:, _SLOTS[k]] = v.to(device=dev, dtype=torch.float32) if torch.is_tensor(v) else v
    return t


class DLADMMNet(_DLADMMBase):
    """V1, main_lena.py:16-102 (also main_syn_l1l1.py, main_syn_gt.py)."""
    VARIANT = _lib.V1_LENA
    GRAD_SLOTS = {"beta1": ("elem1", ()), "beta2": ("elem2", ())}
    PARAM_STEPS = dict(_DLADMMBase.PARAM_STEPS, beta1="zl")   # main_lena.py:85,89

    def _register_params(self):
        # main_lena.py:30-41: beta1/beta2 (m, batch_size) per layer; thresholds are plain tensors
        self.beta1 = nn.ParameterList()
        self.beta2 = nn.ParameterList()
        self.fc = nn.ModuleList()
        for _ in range(self.layers):
            # (m, batch_size); a batch shard holds its own columns only (batch_shard=)
            self.beta1.append(nn.Parameter(torch.ones(self.m, self._pcols, dtype=torch.float32)))
            self.beta2.append(nn.Parameter(torch.ones(self.m, self._pcols, dtype=torch.float32)))
            self.fc.append(nn.Linear(self.m, self.d, bias=False))
        self.active_para = _dev(torch.tensor(0.025, dtype=torch.float32))
        self.active_para1 = _dev(torch.tensor(0.06, dtype=torch.float32))

    def _table_spec(self):
        return {"scalar": dict(thz=self.active_para.float(), the=self.active_para1.float(),
                               s1=1.0)}

    def _elem_param_lists(self) -> list:
        return [self.beta1, self.beta2]

    def _elem_betas(self, cols=None):
        def sl(b):
            b = b.detach()
            # a column shard (training_loss(cols=...)): the backward needs contiguous betas
            return b if cols is None else b[:, cols[0]:cols[1]].contiguous()
        return dict(beta1_elem=[sl(b) for b in self.beta1], beta2_elem=[sl(b) for b in self.beta2])


class DLADMMNetLTheta(_DLADMMBase):
    """V2, main_syn_l1l1_ltheta.py:16-95 (also _bkp, _rw, -dgap, main_syn_gt_ltheta.py)."""
    VARIANT = _lib.V2_LTHETA
    # beta1 serves both Var and L (main_syn_l1l1_ltheta.py:74,80): its grad sums slots b1 + b3
    GRAD_SLOTS = {"beta1": ("row", (_lib.P_BETA1, _lib.P_BETA3)),
                  "beta2": ("row", (_lib.P_BETA2,)),
                  "active_para": ("row", (_lib.P_THETA_Z,)),
                  "active_para1": ("row", (_lib.P_THETA_E,))}
    PARAM_STEPS = dict(_DLADMMBase.PARAM_STEPS, beta1="zl")   # main_syn_l1l1_ltheta.py:74,80

    def _register_params(self):
        # main_syn_l1l1_ltheta.py:30-43
        self._plist("beta1", (self.m, 1), 1.0)
        self._plist("beta2", (self.m, 1), 1.0)
        self._plist("active_para", (self.d, 1), 0.025)
        self._plist("active_para1", (self.m, 1), 0.06)
        self.fc = nn.ModuleList([nn.Linear(self.m, self.d, bias=False) for _ in range(self.layers)])

    def _table_spec(self):
        return {"row": dict(b1=self.beta1, b2=self.beta2, b3=self.beta1, the=self.active_para1,
                            thz=self.active_para)}


class DLADMMNetFull(_DLADMMBase):
    """V3, main_syn_l1l1_full.py:16-96 (also main_syn_l1l1-sl2_full.py)."""
    VARIANT = _lib.V3_FULL
    WSCALE = 0.4
    GRAD_SLOTS = {"beta1": ("row", (_lib.P_BETA1,)), "beta2": ("row", (_lib.P_BETA2,)),
                  "beta3": ("row", (_lib.P_BETA3,)), "ss2": ("row", (_lib.P_SS2,)),
                  "active_para": ("row", (_lib.P_THETA_Z,)),
                  "active_para1": ("row", (_lib.P_THETA_E,))}

    def _register_params(self):
        # main_syn_l1l1_full.py:29-44
        for nm in ("beta1", "beta2", "beta3", "ss2"):
            self._plist(nm, (self.m, 1), 1.0)
        self._plist("active_para", (self.d, 1), 0.2)
        self._plist("active_para1", (self.m, 1), 0.8)
        self.fc = nn.ModuleList([nn.Linear(self.m, self.d, bias=False) for _ in range(self.layers)])

    def _table_spec(self):
        return {"row": dict(b1=self.beta1, b2=self.beta2, b3=self.beta3, ss2=self.ss2,
                            the=self.active_para1, thz=self.active_para)}


class DLADMMNetScalar(_DLADMMBase):
    """V4, main_syn_l1l1_scalar.py:34-131 (also -sl2_scalar, _scalar_z0)."""
    VARIANT = _lib.V4_SCALAR
    RETURNS_T = True
    WSCALE = 0.4
    NAME = "DLADMMNet_scalar"
    GRAD_SLOTS = {"beta1": ("scalar", (_lib.P_BETA1,)), "beta2": ("scalar", (_lib.P_BETA2,)),
                  "beta3": ("scalar", (_lib.P_BETA3,)), "ss2": ("scalar", (_lib.P_SS2,)),
                  "active_para": ("scalar", (_lib.P_THETA_Z,)),
                  "active_para1": ("scalar", (_lib.P_THETA_E,))}

    def __init__(self, m, n, d, batch_size, A, Z0, E0, L0, layers, **kw):
        super().__init__(m, n, d, batch_size, A, Z0, E0, L0, layers, **kw)
        # main_syn_l1l1_scalar.py:41-48 attributes used by the (un-learned) KM iteration
        self.At = self.A.t()
        A_np = A.detach().cpu().numpy()
        self.A_np = A_np
        self.L = _dev((np.linalg.norm(np.matmul(A_np.T, A_np), ord=2) * torch.ones(1, 1)).float())

    def _register_params(self):
        # main_syn_l1l1_scalar.py:50-65
        for nm in ("beta1", "beta2", "beta3", "ss2"):
            self._plist(nm, (1, 1), 1.0)
        self._plist("active_para", (1, 1), 0.2)
        self._plist("active_para1", (1, 1), 0.8)
        self.fc = nn.ModuleList([nn.Linear(self.m, self.d, bias=False) for _ in range(self.layers)])

    def _table_spec(self):
        return {"scalar": dict(b1=self.beta1, b2=self.beta2, b3=self.beta3, ss2=self.ss2,
                               the=self.active_para1, thz=self.active_para, s1=1.0)}


class DLADMMNetScalarSl2(DLADMMNetScalar):
    """V4 as main_syn_l1l1-sl2_scalar.py:17-114 carries it: the same body, but name() returns
    "DLADMMNet" (:113-114), the stem of that script's checkpoints."""
    NAME = "DLADMMNet"


class DLADMMNetScalarZ0(DLADMMNetScalar):
    """V4 as main_syn_l1l1_scalar_z0.py:17-114 carries it (name() "DLADMMNet", :113-114)."""
    NAME = "DLADMMNet"


class DLADMMNetScalarTied(DLADMMNetScalar):
    """V5, main_syn_l1l1_scalar_tied.py:34-104: one shared fc scaled by ss1[k]."""
    VARIANT = _lib.V5_TIED
    NAME = "DLADMMNet_scalar_tied"
    GRAD_SLOTS = dict(DLADMMNetScalar.GRAD_SLOTS, ss1=("scalar", (_lib.P_S1,)))

    def _register_params(self):
        # main_syn_l1l1_scalar_tied.py:50-66 (registration order = state_dict order)
        for nm in ("beta1", "beta2", "beta3", "ss1", "ss2"):
            self._plist(nm, (1, 1), 1.0)
        self._plist("active_para", (1, 1), 1e-4)
        self._plist("active_para1", (1, 1), 1e-2)
        self.fc = nn.Linear(self.m, self.d, bias=False)

    def _weights(self):
        return [self.fc.weight] * self.layers

    def _table_spec(self):
        return {"scalar": dict(b1=self.beta1, b2=self.beta2, b3=self.beta3, ss2=self.ss2,
                               the=self.active_para1, thz=self.active_para, s1=self.ss1)}


class DLADMMNetLasso(DLADMMNetScalar):
    """V6, main_syn_lasso_scalar.py:17-118: E = ss2_1*(X - A Z) - ss2_2*L."""
    VARIANT = _lib.V6_LASSO
    NAME = "DLADMMNet"
    GRAD_SLOTS = {"beta1": ("scalar", (_lib.P_BETA1,)), "beta3": ("scalar", (_lib.P_BETA3,)),
                  "ss2_1": ("scalar", (_lib.P_SS2,)), "ss2_2": ("scalar", (_lib.P_SS2B,)),
                  "active_para": ("scalar", (_lib.P_THETA_Z,))}

    def _register_params(self):
        # main_syn_lasso_scalar.py:33-50
        self._plist("beta1", (1, 1), 1.0)
        self._plist("beta3", (1, 1), 1.0)
        self._plist("ss2_1", (1, 1), 0.5)
        self._plist("ss2_2", (1, 1), 0.5)
        self._plist("active_para", (1, 1), 0.2)
        self.fc = nn.ModuleList([nn.Linear(self.m, self.d, bias=False) for _ in range(self.layers)])

    def _table_spec(self):
        return {"scalar": dict(b1=self.beta1, b3=self.beta3, ss2=self.ss2_1, ss2b=self.ss2_2,
                               thz=self.active_para, s1=1.0)}


class DLADMMNetNewS(DLADMMNetScalar):
    """V7, main_syn_scalar_newS_layerwise.py:34-114: the "new S" layer-wise schedule.

    Its recurrence is V4's with the E/L-step of layer k-1 moved in front of the Z-step of layer
    k (:82-92): newS Z[k] = V4 Z_k, newS E[k] = V4 E_{k-1} (E[0] = E0), newS L[k] = V4 L_{k-1}
    (L[0] = L0), with the same parameters and the same floating-point operations.  So it runs
    as the V4 op over min(K, layers) layers (a schedule flag on the same kernel, SURVEY.md
    section 8 row f4) and re-indexes the outputs; the last layer's E/L-step, which newS never
    uses, is computed and discarded.  forward(x, K) returns (Z, E, L), as the reference."""
    NAME = "DLADMMNet_scalar_newS_layerwise"
    THZ0 = 0.1   # main_syn_scalar_newS_layerwise.py:63-64
    THE0 = 0.1

    def _register_params(self):
        # main_syn_scalar_newS_layerwise.py:51-65
        for nm in ("beta1", "beta2", "beta3", "ss2"):
            self._plist(nm, (1, 1), 1.0)
        self._plist("active_para", (1, 1), self.THZ0)
        self._plist("active_para1", (1, 1), self.THE0)
        self.fc = nn.ModuleList([nn.Linear(self.m, self.d, bias=False) for _ in range(self.layers)])

    def forward(self, x, K=None):
        nl = self.layers if K is None else min(int(K), self.layers)  # :78
        Z, E, L, _T = self._forward_layers(x, nl)
        return Z, [self.E0] + E[: nl - 1], [self.L0] + L[: nl - 1]


class DLADMMNetTiedNewS(DLADMMNetNewS):
    """main_syn_scalar_tied_newS_layerwise.py:34-112: newS schedule, one shared fc scaled by
    ss1[k] (the V5 kernel path)."""
    VARIANT = _lib.V5_TIED
    NAME = "DLADMMNet_scalar_tied_newS_layerwise"
    THZ0 = 0.01
    THE0 = 0.01
    GRAD_SLOTS = dict(DLADMMNetScalar.GRAD_SLOTS, ss1=("scalar", (_lib.P_S1,)))

    def _register_params(self):
        # :51-66 (registration order = state_dict order)
        for nm in ("beta1", "beta2", "beta3", "ss1", "ss2"):
            self._plist(nm, (1, 1), 1.0)
        self._plist("active_para", (1, 1), self.THZ0)
        self._plist("active_para1", (1, 1), self.THE0)
        self.fc = nn.Linear(self.m, self.d, bias=False)

    def _weights(self):
        return [self.fc.weight] * self.layers

    def _table_spec(self):
        return DLADMMNetScalarTied._table_spec(self)


class DLADMMNetPTiedNewS(DLADMMNetTiedNewS):
    """main_syn_scalar_ptied_newS_layerwise.py:34-121: newS schedule with partial weight tying --
    layers // interval weights, layer k uses fc[k // interval] scaled by ss1[k] (:92).
    Constructor adds `interval` (:36)."""
    NAME = "DLADMMNet_scalar_ptied_newS_layerwise"

    def __init__(self, m, n, d, batch_size, A, Z0, E0, L0, layers, interval, **kw):
        self.interval = interval
        super().__init__(m, n, d, batch_size, A, Z0, E0, L0, layers, **kw)

    def _register_params(self):
        # :51-71: fc (layers // interval Linears) is registered after the ParameterLists
        for nm in ("beta1", "beta2", "beta3", "ss1", "ss2"):
            self._plist(nm, (1, 1), 1.0)
        self._plist("active_para", (1, 1), self.THZ0)
        self._plist("active_para1", (1, 1), self.THE0)
        self.fc = nn.ModuleList([nn.Linear(self.m, self.d, bias=False)
                                 for _ in range(self.layers // self.interval)])

    def _weights(self):
        return [self.fc[k // self.interval].weight for k in range(self.layers)]

    def _fc_key(self, k):
        return f"fc.{k // self.interval}.weight"

    def _shared_weight(self):
        return False

    def name(self):
        return "DLADMMNet_scalar_ptied{}_newS_layerwise".format(self.interval)  # :124


VARIANTS = {
    "v1": DLADMMNet, "v2": DLADMMNetLTheta, "v3": DLADMMNetFull,
    "v4": DLADMMNetScalar, "v4_sl2": DLADMMNetScalarSl2, "v4_z0": DLADMMNetScalarZ0,
    "v5": DLADMMNetScalarTied, "v6": DLADMMNetLasso,
    "v7": DLADMMNetNewS, "v7t": DLADMMNetTiedNewS, "v7p": DLADMMNetPTiedNewS,
}


def load_checkpoint(model: nn.Module, path: str, strict: bool = True):
    """`torch.load(model_file); model.load_state_dict(...)` as test_lena_lskm.py:284-285 does,
    accepting a raw state_dict or a {'state_dict': ...} wrapper (the .pth.tar convention).
    Uses weights_only=True: a checkpoint cannot execute code."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    return model.load_state_dict(sd, strict=strict)
