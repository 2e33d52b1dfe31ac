"""The backward as one reverse-sweep kernel (csrc/dladmm_reverse.hip, dladmm_bwd_path() == 1)
against the per-layer backward kernels (flags bwd_per_layer), on the same saved forward.

The reverse kernel forms every product as the per-layer kernels do (one fma chain per output
block, k in the same order) and every elementwise adjoint with the same expressions, so
  * the weight gradients -- built from gU_k and Var_k -- are equal bit for bit;
  * the parameter-slot gradients agree to the rounding of their fp32 per-wave partials (the
    kernels group the terms by wave differently): 2e-6 norm-relative per layer.
Covered: V4 (L1L1 and LASSO objective), V6 and V1 (per-sample betas: their gradients equal bit
for bit too), upstream cotangents of Z, E, L and T, the three register-resident shapes with ragged
rows and columns, K = 1, theta < 0 layers (the shrink masks come from the saved Z_k), a batch
that is not a multiple of 16 (zero padding of the gU / Var rows the weight gradient reads).
Against the reference: tests/test_gpu_backward.py::test_fused_training_loss runs V4 / V6
through this kernel (the fused objective), compared with the reference autograd and the oracle.
"""
from importlib import import_module

import numpy as np
import pytest
import torch

import problems as P
from test_gpu_backward import make_train_net, nrel

pytestmark = pytest.mark.gpu


def saved_forward(dl, variant, m, n, B, K, seed, negtheta=False, lk=0):
    ops = import_module("d-ladmm_amd.ops")
    d = dict(variant=variant, m=m, n=n, B=B, K=K, seed=seed, perturb=0.1, negtheta=negtheta)
    inp, sd = P.build_problem(d)
    net = make_train_net(dl, variant, inp, sd, K).cuda()
    X = torch.from_numpy(inp["X"]).cuda()
    with torch.no_grad():
        tables = net._tables(X.device)
    W = [w.detach() for w in net._weights()]
    args = (net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0)
    with torch.no_grad():
        r = ops.dladmm_forward(*args, keep_all=True, want_T=True, want_P=True, loss_kind=lk,
                               **tables)
    assert r.P is not None
    return ops, args, r, tables


def both(dl, variant, m, n, B, K, seed, kind, flags, negtheta=False):
    lk = dl._lib.LOSS_LASSO if kind == "lasso" else dl._lib.LOSS_L1L1
    ops, args, r, tables = saved_forward(dl, variant, m, n, B, K, seed, negtheta, lk)
    g = torch.Generator(device="cuda").manual_seed(seed)
    coef = (torch.rand(K, 2, device="cuda", generator=g) * torch.tensor([1e-2, 1.0],
                                                                           device="cuda")).contiguous()
    kw = dict(loss_kind=lk, loss_coef=coef, **tables)
    rev = ops.dladmm_backward(*args, r, **kw)
    flags.set(bwd_per_layer=True)
    per = ops.dladmm_backward(*args, r, **kw)
    flags.set(bwd_per_layer=False)
    return rev, per


def check_equal(rev, per, K):
    assert rev.path in (1, 2, 3) and per.path == 0   # 2 / 3: the row-split sweeps (small batches)
    assert torch.equal(rev.gW, per.gW)
    gs_r = rev.g_scalar.cpu().numpy()
    gs_p = per.g_scalar.cpu().numpy()
    from importlib import import_module
    lib = import_module("d-ladmm_amd._lib")
    for k in range(K):
        e = nrel(gs_r[k], gs_p[k])
        assert e <= 2e-6, (k, e, gs_r[k], gs_p[k])
        # the ss1 slot is V5's; s1 is the constant 1 elsewhere and its slot 0 on both paths
        # (also on theta_z < 0 layers, where the per-layer BK2 forms q)
        assert gs_r[k, lib.P_S1] == 0.0 and gs_p[k, lib.P_S1] == 0.0


@pytest.mark.parametrize("variant,kind", [("v4", "l1l1"), ("v4", "lasso"), ("v6", "lasso")])
@pytest.mark.parametrize("shape", [(20, 30, 70, 3), (64, 200, 333, 2), (250, 500, 200, 4),
                                   (256, 512, 64, 1)])
def test_reverse_matches_per_layer(variant, kind, shape, dl, flags):
    m, n, B, K = shape
    rev, per = both(dl, variant, m, n, B, K, 9700 + m, kind, flags)
    check_equal(rev, per, K)


@pytest.mark.parametrize("variant", ["v4", "v6"])
def test_reverse_negative_thresholds(variant, dl, flags):
    """theta_z, theta_e < 0 on every other layer: both relus open where |U| < |theta|; the
    reverse kernel reads S'(U) off the saved Z_k (|Z| < 2|theta| there), the per-layer kernels
    recompute U = Z_{k-1} - W_k Var_k (phase 2)."""
    rev, per = both(dl, variant, 96, 200, 150, 4, 9800, "l1l1", flags, negtheta=True)
    check_equal(rev, per, 4)


def test_reverse_headline_shape_columns(dl, flags):
    """The training bench's shape (V4, m=256, n=512, K=15) at 4,096 columns (64 workgroups)."""
    rev, per = both(dl, "v4", 256, 512, 4096, 15, 9900, "l1l1", flags)
    check_equal(rev, per, 15)


def test_reverse_deterministic(dl):
    ops, args, r, tables = saved_forward(dl, "v4", 64, 200, 333, 3, 9950, lk=dl._lib.LOSS_L1L1)
    coef = torch.tensor([[1e-3, 1.0]] * 3, device="cuda")
    kw = dict(loss_kind=dl._lib.LOSS_L1L1, loss_coef=coef, **tables)
    a = ops.dladmm_backward(*args, r, **kw)
    b = ops.dladmm_backward(*args, r, **kw)
    assert a.path in (1, 2, 3)
    assert torch.equal(a.gW, b.gW) and torch.equal(a.g_scalar, b.g_scalar)


def test_z_cotangents_on_the_reverse_sweep(dl, flags):
    """A torch-op loss over the returned Z_k (the reference's own training loop) hands the
    backward per-layer Z cotangents only: the reverse sweep adds them where the per-layer BK2
    does ((adjoint + gZ_k) + A^T gP), so both paths agree bit for bit on the weight gradients;
    an unread layer's cotangent may be None."""
    ops, args, r, tables = saved_forward(dl, "v4", 64, 200, 333, 3, 9960, lk=dl._lib.LOSS_L1L1)
    g = torch.Generator(device="cuda").manual_seed(9961)
    gz = [torch.randn(200, 333, device="cuda", generator=g), None,
          torch.randn(200, 333, device="cuda", generator=g)]
    coef = torch.tensor([[1e-3, 1.0]] * 3, device="cuda")
    kw = dict(loss_kind=dl._lib.LOSS_L1L1, loss_coef=coef, **tables)
    rev = ops.dladmm_backward(*args, r, gz, **kw)
    flags.set(bwd_per_layer=True)
    per = ops.dladmm_backward(*args, r, gz, **kw)
    flags.set(bwd_per_layer=False)
    check_equal(rev, per, 3)


def _cotangents(m, n, B, K, seed, which):
    """Random upstream cotangents of the outputs named in `which` (subset of "ZELT"), one layer
    of each left None (an output the loss never reads)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    rows = dict(Z=n, E=m, L=m, T=m)
    out = {}
    for nm in "ZELT":
        if nm not in which:
            out[nm] = None
            continue
        cnt = K + 1 if nm == "T" else K
        out[nm] = [None if j == 1 % cnt else
                   torch.randn(rows[nm], B, device="cuda", generator=g) for j in range(cnt)]
    return out


def both_cot(dl, variant, m, n, B, K, seed, flags, which, fused_loss):
    lk = dl._lib.LOSS_L1L1 if fused_loss else 0
    ops, args, r, tables = saved_forward(dl, variant, m, n, B, K, seed, lk=lk)
    c = _cotangents(m, n, B, K, seed + 1, which)
    kw = dict(**tables)
    if fused_loss:
        g = torch.Generator(device="cuda").manual_seed(seed + 2)
        kw.update(loss_kind=lk, loss_coef=(torch.rand(K, 2, device="cuda", generator=g) *
                                           torch.tensor([1e-2, 1.0], device="cuda")).contiguous())
    cots = (c["Z"], c["E"], c["L"], c["T"])
    rev = ops.dladmm_backward(*args, r, *cots, **kw)
    flags.set(bwd_per_layer=True)
    per = ops.dladmm_backward(*args, r, *cots, **kw)
    flags.set(bwd_per_layer=False)
    return rev, per


@pytest.mark.parametrize("variant", ["v4", "v6"])
@pytest.mark.parametrize("shape", [(20, 30, 70, 3), (250, 500, 200, 4)])
def test_elt_cotangents_on_the_reverse_sweep(variant, shape, dl, flags):
    """Cotangents of E_k, L_k and T_k (a loss over every returned list) join the sweep in round
    4: added to the incoming adjoints of BK1 where the per-layer kernels add them, so the two
    paths agree bit for bit on the weight gradients (with the fused objective too)."""
    m, n, B, K = shape
    for which, fused in (("ZELT", False), ("ELT", True), ("L", False)):
        rev, per = both_cot(dl, variant, m, n, B, K, 9970 + m, flags, which, fused)
        check_equal(rev, per, K)


def check_equal_v1(rev, per, K):
    assert rev.path in (1, 2, 3) and per.path == 0   # 2 / 3: the row-split sweeps (small batches)
    assert rev.g_scalar is None and per.g_scalar is None
    assert torch.equal(rev.gW, per.gW)
    for k in range(K):
        assert torch.equal(rev.g_beta1[k], per.g_beta1[k]), f"g_beta1[{k}]"
        assert torch.equal(rev.g_beta2[k], per.g_beta2[k]), f"g_beta2[{k}]"


@pytest.mark.parametrize("shape", [(20, 30, 70, 3), (64, 200, 333, 2), (250, 500, 200, 4),
                                   (256, 512, 64, 1)])
@pytest.mark.parametrize("loss", ["lena", "fused", "zonly"])
def test_reverse_v1_matches_per_layer(shape, loss, dl, flags):
    """V1 (main_lena.py:57-98, per-sample betas) on the reverse sweep: its betas and their
    gradients are per-element operands of the G2' rows; beta1's gradient sums BK1's term (one
    pass) and BK3's (the next) in the per-layer sweep's order.  Losses: main_lena.py:221-228's
    (cotangents of Z, E and L), the fused L1L1 objective, a Z-only torch loss.  Weight and
    beta gradients equal the per-layer path's bit for bit."""
    m, n, B, K = shape
    which, fused = {"lena": ("ZEL", False), "fused": ("", True), "zonly": ("Z", False)}[loss]
    rev, per = both_cot(dl, "v1", m, n, B, K, 9990 + m, flags, which, fused)
    check_equal_v1(rev, per, K)


def test_reverse_v1_headline_shape(dl, flags):
    """V1 at m=256, n=512, K=15 on 4,096 columns with the main_lena.py loss's cotangents."""
    rev, per = both_cot(dl, "v1", 256, 512, 4096, 15, 9995, flags, "ZEL", False)
    check_equal_v1(rev, per, 15)


def _zmask_ab(dl, variant, m, n, B, K, seed, flags, mixed=False):
    """The per-row-theta variants' BK2 with masks read off the saved Z_k (PH 5) against the
    recomputing BK2 (PH 2, flags bwd_no_zmask).  mixed: theta_z of every other ROW negative in
    every layer (each row takes its own branch of the mask)."""
    ops = import_module("d-ladmm_amd.ops")
    d = dict(variant=variant, m=m, n=n, B=B, K=K, seed=seed, perturb=0.1, negtheta=not mixed)
    inp, sd = P.build_problem(d)
    if mixed:
        for k in range(K):
            key = f"active_para.{k}"
            v = sd[key].copy()
            v[1::2] = -0.3 * np.abs(v[1::2])
            sd[key] = v
    net = make_train_net(dl, variant, inp, sd, K).cuda()
    X = torch.from_numpy(inp["X"]).cuda()
    with torch.no_grad():
        tables = net._tables(X.device)
    W = [w.detach() for w in net._weights()]
    args = (net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0)
    lk = dl._lib.LOSS_L1L1
    with torch.no_grad():
        r = ops.dladmm_forward(*args, keep_all=True, want_T=True, want_P=True, loss_kind=lk,
                               **tables)
    coef = torch.tensor([[1e-2, 1.0]] * K, device="cuda")
    kw = dict(loss_kind=lk, loss_coef=coef, **tables)
    a = ops.dladmm_backward(*args, r, **kw)
    flags.set(bwd_no_zmask=True)
    b = ops.dladmm_backward(*args, r, **kw)
    flags.set(bwd_no_zmask=False)
    assert nrel(a.gW.cpu().numpy(), b.gW.cpu().numpy()) <= 1e-6
    ga, gb = a.g_row.cpu().numpy(), b.g_row.cpu().numpy()
    for k in range(K):
        assert nrel(ga[k], gb[k]) <= 1e-6, k


@pytest.mark.parametrize("variant", ["v2", "v3"])
@pytest.mark.parametrize("mixed", [False, True])
def test_per_row_theta_zmask_matches_recomputing(variant, mixed, dl, flags):
    """negtheta (mixed=False): theta < 0 on every other layer; mixed: on every other row."""
    _zmask_ab(dl, variant, 96, 200, 150, 4, 9870, flags, mixed)


@pytest.mark.parametrize("tied", [False, True])
def test_reverse_v5_tied_step(tied, dl, flags):
    """V5 (one shared weight, a trainable step ss1_k on W Var_k) on the reverse sweep: ss1_k's
    gradient -<W, gU_k Var_k^T> from the weight gradient's sums in both paths; the per-layer
    path's BK2 reads the masks off Z_k too.  gW summed over the layers (tied) or per layer."""
    ops, args, r, tables = saved_forward(dl, "v5", 64, 200, 333, 4, 9990, lk=dl._lib.LOSS_L1L1)
    coef = torch.tensor([[1e-2, 1.0]] * 4, device="cuda")
    kw = dict(loss_kind=dl._lib.LOSS_L1L1, loss_coef=coef, tied=tied, **tables)
    rev = ops.dladmm_backward(*args, r, **kw)
    flags.set(bwd_per_layer=True)
    per = ops.dladmm_backward(*args, r, **kw)
    flags.set(bwd_per_layer=False)
    assert rev.path in (1, 2, 3) and per.path == 0   # 2 / 3: the row-split sweeps (small batches)
    assert torch.equal(rev.gW, per.gW)
    gs_r, gs_p = rev.g_scalar.cpu().numpy(), per.g_scalar.cpu().numpy()
    for k in range(4):
        assert nrel(gs_r[k], gs_p[k]) <= 2e-6, (k, gs_r[k], gs_p[k])
    assert np.all(gs_r[:, 7] != 0.0)  # the ss1 slot (P_S1) is filled


def check_equal_row(rev, per, K):
    """V2 / V3: weight gradients bit for bit; the per-row parameter gradients are the same fp32
    per-wave partials (row16_sum of the same elements) reduced in the same fixed fp64 order --
    except BK1 of the last layer, whose per-layer kernel (phase 4, no GEMM) groups a row's terms
    by 64 columns instead of 16: 2e-6 norm-relative, the bar of the scalar slots above."""
    assert rev.path in (1, 2, 3) and per.path == 0   # 2 / 3: the row-split sweeps (small batches)
    assert torch.equal(rev.gW, per.gW)
    gr, gp = rev.g_row.cpu().numpy(), per.g_row.cpu().numpy()
    assert gr.shape == gp.shape
    for k in range(K):
        e = nrel(gr[k], gp[k])
        assert e <= (2e-6 if k == K - 1 else 1e-12), (k, e)


@pytest.mark.parametrize("variant", ["v2", "v3"])
@pytest.mark.parametrize("shape", [(20, 30, 70, 3), (64, 200, 333, 2), (250, 500, 200, 4),
                                   (256, 512, 64, 1)])
@pytest.mark.parametrize("loss", ["fused", "zel"])
def test_reverse_per_row_params(variant, shape, loss, dl, flags):
    """V2 (main_syn_l1l1_ltheta.py) and V3 (main_syn_l1l1_full.py) on the reverse sweep (round
    4): per-row parameters as row-table operands, per-row gradient partials per (layer, slot,
    row, 16-column wave) as the per-layer kernels form them."""
    m, n, B, K = shape
    which, fused = {"fused": ("", True), "zel": ("ZEL", False)}[loss]
    rev, per = both_cot(dl, variant, m, n, B, K, 9870 + m, flags, which, fused)
    check_equal_row(rev, per, K)


@pytest.mark.parametrize("variant", ["v2", "v3"])
def test_reverse_per_row_headline_shape(variant, dl, flags):
    rev, per = both_cot(dl, variant, 256, 512, 4096, 15, 9880, flags, "", True)
    check_equal_row(rev, per, 15)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["v2", "v3"])
def test_per_row_negative_theta_masks_at_the_boundary(variant, dl):
    """Per-row theta_z < 0 with U = Z_{k-1} - W Var placed exactly at -|theta| and one ulp either
    side (W_0 = 0, so U = Z0 exactly): the reverse sweep reads S'(U) off the saved Z_k, which the
    forward forms in the clamp form (Z = 2U exactly where both relus are open).  Against fp64
    autograd of the reference-op restatement (literal two-relu shrink, torch's relu'(0) = 0):
    theta_z's per-row gradient is a sum of +-cotangents, so a dropped or extra mask term shows
    as an O(1) relative error."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "oracle"))
    import dladmm_torch_cpu as TC
    m, n, B, K = 32, 64, 64, 1
    inp = P.make_inputs(m, n, B, 9910)
    sd = P.make_state_dict(variant, m, n, B, K, inp["A"], 9910, perturb=0.1)
    c = np.linspace(0.05, 0.3, n).astype(np.float32)           # |theta| per row
    sd["active_para.0"] = (-c).reshape(n, 1)
    sd["fc.0.weight"] = np.zeros_like(sd["fc.0.weight"])        # U = Z0 exactly
    Z0 = np.empty((n, B), np.float32)
    picks = []
    for i in range(n):
        ci = np.float32(c[i])
        picks.append([-ci, np.nextafter(-ci, np.float32(-1)), np.nextafter(-ci, np.float32(1)),
                      ci, np.nextafter(ci, np.float32(1)), np.nextafter(ci, np.float32(-1)),
                      np.float32(0.0), -2 * ci])
    for b in range(B):
        Z0[:, b] = [picks[i][b % 8] for i in range(n)]
    inp = dict(inp, Z0=Z0)
    G = np.random.default_rng(9911).standard_normal((n, B)).astype(np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    net = dl.VARIANTS[variant](m=m, n=0, d=n, batch_size=B, A=t(inp["A"]), Z0=t(Z0),
                               E0=t(inp["E0"]), L0=t(inp["L0"]), layers=K)
    net.load_state_dict({k: t(v) for k, v in sd.items()}, strict=True)
    net = net.cuda().requires_grad_(True)
    out = net(t(inp["X"]).cuda())
    (out[0][0] * t(G).cuda()).sum().backward()
    g_gpu = net.active_para[0].grad.detach().cpu().double().numpy().ravel()
    d64 = lambda a: torch.from_numpy(np.asarray(a, np.float64))  # noqa: E731
    params = {k: d64(v).requires_grad_(True) for k, v in sd.items()}
    fwd = getattr(TC.forward, "__wrapped__", TC.forward)
    with torch.enable_grad():
        o64 = fwd(variant, d64(inp["X"]), d64(inp["A"]), d64(Z0), d64(inp["E0"]),
                  d64(inp["L0"]), params, K)
        (o64[0][0] * d64(G)).sum().backward()
    g64 = params["active_para.0"].grad.numpy().ravel()
    assert np.allclose(g_gpu, g64, rtol=1e-5, atol=1e-5 * np.abs(g64).max()), \
        np.abs(g_gpu - g64).max()
