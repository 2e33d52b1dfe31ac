"""Paths 5 and 6, the small-batch row-split forms of the fused forward: path 5
(csrc/dladmm_fused_rs.hip) a workgroup per 16 batch columns, each product's output rows split
over its 4 waves; path 6 (csrc/dladmm_fused_xs.hip) four workgroups per 16 columns, the rows over
their 16 waves, the column state handed between the workgroups through global memory once per
product.  Each test runs both: split "xs" = the default plan (path 6 where its grid fits one
workgroup per CU, B <= 1,024 on 256 CUs), "rs" = plan flag no_xsplit (path 5).

It performs the fused kernel's arithmetic operation for operation, so its outputs must equal
path 1's (plan flag no_rowsplit) BIT FOR BIT -- every layer's Z, E, L and T -- for V4, V5 (and
the KM iteration of the test scripts built on V5) and V6, at ragged batches and shapes, lean and
keep_all; one case is also checked against the oracle at the fp32 bar directly.  The plan takes
path 5 where it applies (V1 / V4 / V5 / V6 at the 256 x 512 shape, fp32, at most three 16-column
workgroups per CU), training forwards included: their saved products bit for bit, the fused
objective to fp32 rounding."""
import numpy as np
import pytest
import torch

import problems as P
from test_gpu_parity import _compare, _oracle_case

pytestmark = pytest.mark.gpu


# the scalar-parameter slots of the row-split sweeps against the 64-column sweep: the same terms
# summed in another order (per-wave partials over a quarter -- bwd path 3: a sixteenth -- of the
# rows, then fp64 over the waves); slots such as theta_z's sum terms that cancel, so two fp32
# orders differ by up to ~2e-6 of the slot vector's norm.  1e-5 is the fp32 bar of the parity
# tests.
PSLOT_TOL = 1e-5


def _cus():
    return torch.cuda.get_device_properties(0).multi_processor_count


def _xs_grid(B):
    """dladmm_fused_xs.hip xs_grid: four workgroups per 16-column group, groups padded to 8."""
    groups = -(-B // 16)
    return -(-groups // 8) * 8 * 4


def _split(dl, split, B):
    """(plan flags, expected forward path) of a row-split flavour at batch B."""
    if split == "rs":
        return dl._lib.F_NO_XSPLIT, 5
    return 0, (6 if _xs_grid(B) <= _cus() else 5)


def _run(dl, variant, inp, sd, K, keep_all=True, flags=0, **kw):
    ops = dl.ops
    m, n = inp["A"].shape
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    cls = dl.VARIANTS[variant]
    net = cls(m=m, n=0, d=n, batch_size=inp["X"].shape[1], A=t(inp["A"]), Z0=t(inp["Z0"]),
              E0=t(inp["E0"]), L0=t(inp["L0"]), layers=K)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    net.cuda().requires_grad_(False)
    X = t(inp["X"])
    with torch.no_grad():
        tables = net._tables(X.device)
        W = [w.detach() for w in net._weights()]
        r = ops.dladmm_forward(net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0,
                               keep_all=keep_all, want_T=True, flags=flags, **tables, **kw)
    torch.cuda.synchronize()
    return r


@pytest.mark.parametrize("split", ["xs", "rs"])
@pytest.mark.parametrize("variant", ["v1", "v4", "v5", "v6"])
@pytest.mark.parametrize("B", [1, 20, 77, 300, 1000])
def test_rowsplit_bit_equal_to_fused(variant, B, split, dl):
    m, n, K = 250, 500, 6
    d = dict(variant=variant, m=m, n=n, B=B, K=K, seed=5100 + B, perturb=0.2,
             wscale=0.4 if variant == "v1" else P.VARIANT_SPECS[variant]["wscale"])
    inp, sd = P.build_problem(d)
    fl, want = _split(dl, split, B)
    rs = _run(dl, variant, inp, sd, K, flags=fl)
    fu = _run(dl, variant, inp, sd, K, flags=dl._lib.F_NO_ROWSPLIT)
    assert rs.path == want and fu.path == 1
    for nm in ("Z", "E", "L", "T"):
        a, b = getattr(rs, nm), getattr(fu, nm)
        assert a.shape == b.shape, nm
        assert torch.equal(a, b), (nm, float((a - b).abs().max()))


@pytest.mark.parametrize("split", ["xs", "rs"])
@pytest.mark.parametrize("shape", [(256, 512), (100, 300), (65, 257)])
def test_rowsplit_shapes_and_lean_mode(shape, split, dl):
    """Ragged m / n inside the 256 x 512 instantiation (padded rows stay zero), lean mode (last
    layer only), against path 1 bit for bit."""
    m, n = shape
    K, B = 4, 45
    d = dict(variant="v4", m=m, n=n, B=B, K=K, seed=5200 + m, perturb=0.2, wscale=0.4)
    inp, sd = P.build_problem(d)
    fl, want = _split(dl, split, B)
    for keep_all in (True, False):
        rs = _run(dl, "v4", inp, sd, K, keep_all=keep_all, flags=fl)
        fu = _run(dl, "v4", inp, sd, K, keep_all=keep_all, flags=dl._lib.F_NO_ROWSPLIT)
        assert rs.path == want and fu.path == 1
        for nm in ("Z", "E", "L", "T"):
            assert torch.equal(getattr(rs, nm), getattr(fu, nm)), (keep_all, nm)


@pytest.mark.parametrize("split", ["xs", "rs"])
@pytest.mark.parametrize("variant", ["v1", "v4", "v6"])
@pytest.mark.parametrize("B", [20, 25, 300])
def test_rowsplit_training_forward(variant, B, split, dl):
    """A training forward on path 5 (the reference loops' batches of 20 / 25): the saved
    products P_k = A Z_k bit for bit with path 1's, the fused objective's per-layer sums and
    per-column terms to fp32 rounding (each wave sums a quarter of the rows, then the quarters)."""
    m, n, K = 250, 500, 5
    d = dict(variant=variant, m=m, n=n, B=B, K=K, seed=5150 + B, perturb=0.2,
             wscale=0.4 if variant == "v1" else P.VARIANT_SPECS[variant]["wscale"])
    inp, sd = P.build_problem(d)
    L = dl._lib
    kind = L.LOSS_LASSO if variant == "v6" else L.LOSS_L1L1
    kw = dict(want_P=True, loss_kind=kind, want_col_loss=True)
    fl, want = _split(dl, split, B)
    rs = _run(dl, variant, inp, sd, K, flags=fl, **kw)
    fu = _run(dl, variant, inp, sd, K, flags=L.F_NO_ROWSPLIT, **kw)
    assert rs.path == want and fu.path == 1
    for nm in ("Z", "E", "L", "T", "P"):
        assert torch.equal(getattr(rs, nm), getattr(fu, nm)), nm
    # 1e-5: the fused objective's bar elsewhere (test_gpu_configs objective_vs_reduction)
    np.testing.assert_allclose(rs.loss_sums.cpu().numpy(), fu.loss_sums.cpu().numpy(),
                               rtol=1e-5)
    np.testing.assert_allclose(rs.col_loss.cpu().numpy(), fu.col_loss.cpu().numpy(),
                               rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("split", ["xs", "rs"])
def test_rowsplit_vs_oracle(split, dl, oracle):
    """Independent of path 1: the oracle at the fp32 bar, V4 at m=250 n=500 K=15, B=100."""
    m, n, K, B = 250, 500, 15, 100
    inp, sd, ref = _oracle_case(oracle, "v4", m, n, B, K, seed=5300)
    fl, want = _split(dl, split, B)
    r = _run(dl, "v4", inp, sd, K, flags=fl)
    assert r.path == want
    _compare((list(r.Z), list(r.E), list(r.L), list(r.T)), ref, tag=f"rowsplit {split} v4 B=100",
             path="f32")


def test_km_ground_truth_on_rowsplit(dl):
    """The test scripts' KM ground truth (V5, W = A^T shared, K iterations) at m=250 n=500, B=20:
    paths 6 and 5 equal path 1 bit for bit over 300 iterations."""
    from test_gpu_lskm import make
    d = dict(variant="v4", m=250, n=500, B=20, K=3, seed=5400, perturb=0.1)
    inp, sd = P.build_problem(d)
    case = dict(layers=3, alpha=0.01, delta=-99.0, mu="None", mu_param=0.0)
    net = make(dl, case, inp, sd)
    X = torch.from_numpy(inp["X"]).cuda()
    ops = dl.ops
    Z, E, L, T = net(X, False, False, False, K=300)
    with ops.plan_flags(no_xsplit=True):
        Z5, E5, L5, T5 = net(X, False, False, False, K=300)
    with ops.plan_flags(no_rowsplit=True):
        Zf, Ef, Lf, Tf = net(X, False, False, False, K=300)
    for a, a5, b in zip(Z + E + L + T, Z5 + E5 + L5 + T5, Zf + Ef + Lf + Tf):
        assert torch.equal(a, b)
        assert torch.equal(a5, b)


def test_rowsplit_plan_scope(dl):
    """Path 6 where its grid fits one workgroup per CU, path 5 up to three 16-column workgroups
    per CU, for V1 / V4 / V5 / V6 at the 256 x 512 shape, inference or training (fused
    objective, saved product); fp32 only."""
    L = dl._lib
    m, n, K = 250, 500, 3
    cus = torch.cuda.get_device_properties(0).multi_processor_count

    def path(variant="v4", B=64, loss=0, P_=False, mn=(m, n), flags=0):
        d = dict(variant=variant, m=mn[0], n=mn[1], B=B, K=K, seed=5500, perturb=0.1)
        inp, sd = P.build_problem(d)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
        cls = dl.VARIANTS[variant]
        net = cls(m=mn[0], n=0, d=mn[1], batch_size=B, A=t(inp["A"]), Z0=t(inp["Z0"]),
                  E0=t(inp["E0"]), L0=t(inp["L0"]), layers=K).cuda()
        r = dl.ops.dladmm_forward(net.VARIANT, t(inp["X"]), net.A,
                                  [w.detach() for w in net._weights()], net.Z0, net.E0, net.L0,
                                  loss_kind=loss, want_P=P_, flags=flags,
                                  **net._tables(net.A.device))
        return r.path
    assert path() == 6
    assert path(flags=L.F_NO_XSPLIT) == 5
    assert path(variant="v5") == 6 and path(variant="v6") == 6
    xs_max = cus // 32 * 8 * 16   # the largest batch whose padded xs grid fits the CUs
    assert path(B=xs_max) == 6 and path(B=xs_max + 1) == 5
    assert path(B=48 * cus) == 5
    assert path(B=48 * cus + 1) == 1
    assert path(loss=L.LOSS_L1L1) == 6
    assert path(P_=True) == 6
    assert path(variant="v1") == 6
    assert path(variant="v2") == 1 and path(variant="v3") == 1   # per-row parameters
    assert path(mn=(64, 128)) == 1   # the 64 x 256 instantiation: whole-row waves


@pytest.mark.parametrize("variant,kind", [("v4", "l1l1"), ("v4", "lasso"), ("v5", "l1l1"),
                                          ("v6", "lasso")])
@pytest.mark.parametrize("B", [20, 25, 300])
@pytest.mark.parametrize("gz", [False, True])
@pytest.mark.parametrize("split", ["xs", "rs"])
def test_rowsplit_reverse_sweep(variant, kind, B, gz, split, dl):
    """dladmm_bwd_path 2 (the row-split reverse sweep after a path-5 forward) against the reverse
    sweep after a path-1 forward (plan flag no_rowsplit), same saved state: the weight gradients
    bit for bit (from bit-equal gU_k / Var_k), the parameter slots within PSLOT_TOL per layer
    (the per-wave partials cover other element sets), with the fused objective or with Z
    cotangents (a torch-op loss over the returned Z_k, the reference's own training loop)."""
    from test_gpu_backward import make_train_net, nrel
    ops = dl.ops
    L = dl._lib
    m, n, K = 250, 500, 4
    d = dict(variant=variant, m=m, n=n, B=B, K=K, seed=5600 + B, perturb=0.1)
    inp, sd = P.build_problem(d)
    net = make_train_net(dl, variant, inp, sd, K).cuda()
    X = torch.from_numpy(inp["X"]).cuda()
    with torch.no_grad():
        tables = net._tables(X.device)
    W = [w.detach() for w in net._weights()]
    args = (net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0)
    lk = L.LOSS_LASSO if kind == "lasso" else L.LOSS_L1L1
    g = torch.Generator(device="cuda").manual_seed(B)
    coef = (torch.rand(K, 2, device="cuda", generator=g) *
            torch.tensor([1e-2, 1.0], device="cuda")).contiguous()
    out = {}
    xf, _ = _split(dl, split, B)
    for fl in (xf, L.F_NO_ROWSPLIT):
        with torch.no_grad():
            r = ops.dladmm_forward(*args, keep_all=True, want_T=True, want_P=True, loss_kind=lk,
                                   flags=fl, **tables)
        if gz:
            gZ = [torch.randn(n, B, generator=g, device="cuda") / B for _ in range(K)]
            kw = dict(gZ=gZ, **tables)
        else:
            kw = dict(loss_kind=lk, loss_coef=coef, **tables)
        out[fl] = (r.path, ops.dladmm_backward(*args, r, **kw))
        g.manual_seed(B)   # the same cotangents / coefficients for both
        coef = (torch.rand(K, 2, device="cuda", generator=g) *
                torch.tensor([1e-2, 1.0], device="cuda")).contiguous()
    (fp, rs), (fp1, cl) = out[xf], out[L.F_NO_ROWSPLIT]
    assert fp in (5, 6) and fp1 == 1 and rs.path == fp - 3 and cl.path == 1
    assert torch.equal(rs.gW, cl.gW)
    gs_r, gs_c = rs.g_scalar.cpu().numpy(), cl.g_scalar.cpu().numpy()
    for k in range(K):
        assert nrel(gs_r[k], gs_c[k]) <= PSLOT_TOL, (k, gs_r[k], gs_c[k])


@pytest.mark.parametrize("variant,kind", [("v1", "l1l1"), ("v4", "l1l1"), ("v6", "lasso")])
@pytest.mark.parametrize("B", [20, 300])
@pytest.mark.parametrize("cot", ["elt", "all"])
@pytest.mark.parametrize("split", ["xs", "rs"])
def test_rowsplit_reverse_sweep_cotangents(variant, kind, B, cot, split, dl):
    """The row-split reverse sweep with cotangents of E_k / L_k / T_k (main_lena.py:221-228 reads
    E and L; "all" adds Z's) and V1's per-sample betas, against the reverse sweep after a path-1
    forward: weight gradients and V1's beta gradients (per-element stores) bit for bit, the
    scalar-parameter slots within PSLOT_TOL per layer."""
    from test_gpu_backward import make_train_net, nrel
    ops = dl.ops
    L = dl._lib
    m, n, K = 250, 500, 4
    d = dict(variant=variant, m=m, n=n, B=B, K=K, seed=5700 + B, perturb=0.1)
    inp, sd = P.build_problem(d)
    net = make_train_net(dl, variant, inp, sd, K).cuda()
    X = torch.from_numpy(inp["X"]).cuda()
    with torch.no_grad():
        tables = net._tables(X.device)
    W = [w.detach() for w in net._weights()]
    args = (net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0)
    lk = L.LOSS_LASSO if kind == "lasso" else L.LOSS_L1L1
    out = {}
    xf, _ = _split(dl, split, B)
    for fl in (xf, L.F_NO_ROWSPLIT):
        with torch.no_grad():
            r = ops.dladmm_forward(*args, keep_all=True, want_T=True, want_P=True, loss_kind=lk,
                                   flags=fl, **tables)
        g = torch.Generator(device="cuda").manual_seed(B)
        rnd = lambda rows, cnt: [torch.randn(rows, B, generator=g, device="cuda") / B  # noqa: E731
                                 for _ in range(cnt)]
        gE, gL, gT = rnd(m, K), rnd(m, K), rnd(m, r.T.shape[0])
        gZ = rnd(n, K) if cot == "all" else None
        out[fl] = (r.path, ops.dladmm_backward(*args, r, gZ=gZ, gE=gE, gL=gL, gT=gT, **tables))
    (fp, rs), (fp1, cl) = out[xf], out[L.F_NO_ROWSPLIT]
    assert fp in (5, 6) and fp1 == 1 and rs.path == fp - 3 and cl.path == 1
    assert torch.equal(rs.gW, cl.gW)
    if variant == "v1":
        for a, b in zip(rs.g_beta1 + rs.g_beta2, cl.g_beta1 + cl.g_beta2):
            assert torch.equal(a, b)
    else:
        gs_r, gs_c = rs.g_scalar.cpu().numpy(), cl.g_scalar.cpu().numpy()
        for k in range(K):
            assert nrel(gs_r[k], gs_c[k]) <= PSLOT_TOL, (k, gs_r[k], gs_c[k])
