"""Parity of the HIP backward (dladmm_bwd_f32 through the drop-in modules' autograd) with the
reference's own autograd gradients and with the backward oracle.

* golden gradient fixtures (tests/golden/grad_*.npz): the reference classes' `.grad` after
  `total_loss.backward()` with the training loss of main_syn_l1l1_scalar.py:283-298 /
  main_syn_lasso_scalar.py:270-285 plus seeded linear terms on every output -- every variant;
  the loss is built here with torch ops on the GPU outputs, exactly as the reference loops do;
* the same through the per-layer kernel path (flags per_layer);
* the oracle (oracle/dladmm_oracle_grad.py, pinned by those fixtures) at a larger ragged batch;
* determinism (bitwise) and one full Adam training step.

The golden-gradient and fused-objective tests run at both training precisions: "f32" (fp32 MFMA)
and "f32_split" (the split-f16 forward that saves A Z_k, then the reverse sweep with the
split-f16 weight gradient -- the bench's train.split_f16 leg), each against the reference
autograd fixtures at the same GTOL.  Every checked error is logged (tests/parity.py) so a
DLADMM_PARITY_JSON run records the margins.

Tolerance: norm-relative per parameter <= max(GTOL, 3 x the reference's fp32-vs-fp64 gap of that
gradient).  GTOL = 1e-4: the GPU forward sums its GEMMs in another order than CPU BLAS, and a
shrink mask that flips on a near-threshold element moves a gradient by more than fp32 rounding
(the reference's own fp64 twin shows the same effect: its gap column).
"""
from importlib import import_module

import numpy as np
import pytest
import torch

from conftest import load_golden
import parity
import problems as P

pytestmark = pytest.mark.gpu

GTOL = 1e-4


def nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / nb) if nb > 0 else float(np.linalg.norm(a))


# variants whose fused forward has a split-f16 form (csrc/dladmm_fused_x3.hip: V4-V6 and the
# newS schedules built on them); the others train f32 under "f32_split"
SPLIT_VARIANTS = ("v1", "v4", "v5", "v6", "v7", "v7t", "v7p")
PRECISIONS = ("f32", "f32_split")


def make_train_net(dl, variant, inp, sd, K, precision="f32", **extra):
    m, n = inp["A"].shape
    B = inp["X"].shape[1]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    net = dl.VARIANTS[variant](m=m, n=0, d=n, batch_size=B, A=t(inp["A"]), Z0=t(inp["Z0"]),
                               E0=t(inp["E0"]), L0=t(inp["L0"]), layers=K, **extra)
    net.load_state_dict({k: t(v) for k, v in sd.items()}, strict=True)
    net.requires_grad_(True)
    net.precision = precision
    return net


def split_expected(d) -> bool:
    """Whether a "f32_split" training forward of problem d runs the split-f16 kernel (path 4):
    split variants at the register-resident shapes with a batch that is a multiple of 4."""
    return d["variant"] in SPLIT_VARIANTS and d["m"] <= 256 and d["n"] <= 512 and d["B"] % 4 == 0


def record_paths(monkeypatch):
    """The kernel path of every forward the model runs (ForwardResult.path), in call order."""
    mod = import_module("d-ladmm_amd.model")
    orig, paths = mod.dladmm_forward, []

    def wrap(*a, **k):
        r = orig(*a, **k)
        paths.append(r.path)
        return r
    monkeypatch.setattr(mod, "dladmm_forward", wrap)
    return paths


def grad_cases(names):
    """(fixture, precision) pairs: every fixture at f32, the split-f16 ones also at f32_split."""
    out = []
    for nm in names:
        out.append((nm, "f32"))
        if P.grad_defn(P.GRAD_FIXTURES[nm])["variant"] in SPLIT_VARIANTS:
            out.append((nm, "f32_split"))
    return out


def total_loss(out, X, A, up, kind, K):
    """main_syn_l1l1_scalar.py:283-296 (decay 0.6**epoch) + the fixture's linear terms."""
    Z, E, L = out[0], out[1], out[2]
    coeffs = P.loss_coeffs(K)
    alpha = P.GRAD_ALPHA
    tot = 0
    for k in range(K):
        if kind == "l1l1":
            lk = alpha * torch.sum(torch.abs(Z[k]), dim=0).mean() + \
                torch.sum(torch.abs(X - torch.mm(A, Z[k])), dim=0).mean()
        else:
            lk = alpha * torch.sum(torch.abs(Z[k]), dim=0).mean() + \
                0.5 * torch.sum((X - torch.mm(A, Z[k])) ** 2.0, dim=0).mean()
        tot = tot + lk * coeffs[k]
    c = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    for k in range(K):
        tot = tot + (c(up["Gz"][k]) * Z[k]).sum() + (c(up["Ge"][k]) * E[k]).sum() + \
            (c(up["Gl"][k]) * L[k]).sum()
    if "Gt" in up:
        for j in range(K + 1):
            tot = tot + (c(up["Gt"][j]) * out[3][j]).sum()
    return tot


def run_grads(dl, name, precision="f32"):
    g, meta = load_golden(name)
    d = meta["defn"]
    inp, sd = P.build_problem(d)
    up = P.make_upstream(d, P.VARIANT_SPECS[d["variant"]]["ret_t"])
    net = make_train_net(dl, d["variant"], inp, sd, d["K"], precision=precision,
                         **P.ctor_extra(d))
    X = torch.from_numpy(inp["X"]).cuda()
    A = torch.from_numpy(inp["A"]).cuda()
    out = net(X)
    loss = total_loss(out, X, A, up, meta["gdef"]["loss"], d["K"])
    loss.backward()
    torch.cuda.synchronize()
    return g, meta, net, float(loss.detach())


def none_keys(name, which):
    """Parameters whose .grad the reference autograd leaves None for fixture `name`:
    which = 'fixture_loss' (the fixture's loss) or 'training_loss' (the bare training loss over
    the Z's), recorded by make_golden_grad.py --none-keys from the reference classes."""
    import json
    import os
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "grad_none_keys.json")) as f:
        return set(json.load(f)[name][which])


def check_against_golden(g, meta, net, path="f32"):
    got = {k: p.grad for k, p in net.named_parameters()}
    worst = {}
    none = none_keys(meta["name"], "fixture_loss")
    for key in meta["keys"]:
        assert (got[key] is None) == (key in none), key
        if got[key] is None:
            continue
        ref = g["g:" + key]
        e = nrel(got[key].detach().cpu().numpy(), ref)
        gap = float(g["gap:" + key])
        tol = max(GTOL, 3.0 * gap)
        worst[key] = e
        parity.check(meta["name"] + " grad vs reference autograd", path, key, e, tol, gap)
    return worst


@pytest.mark.parametrize("name,precision", grad_cases(sorted(P.GRAD_FIXTURES)))
def test_grads_match_reference_autograd(name, precision, dl, monkeypatch):
    """The reference's own autograd gradients (golden fixtures) at both training precisions;
    under "f32_split" the forward must have run the split-f16 kernel wherever it applies (and
    then the backward's weight gradient runs split-f16 too)."""
    paths = record_paths(monkeypatch)
    g, meta, net, loss = run_grads(dl, name, precision)
    assert paths, "no forward ran"
    if precision == "f32_split":
        assert paths[0] == (4 if split_expected(meta["defn"]) else 1), paths
    np.testing.assert_allclose(loss, g["loss"][0], rtol=1e-4)
    check_against_golden(g, meta, net, path=precision)


@pytest.mark.parametrize("name", ["grad_v4_med", "grad_v6_med", "grad_v1_med", "grad_v3_med",
                                  "grad_v5_small", "grad_v2_ragged"])
def test_grads_layered_path(name, dl, flags):
    """Forward and backward both on the per-layer kernels (the path of m > 256 / n > 512)."""
    flags.set(per_layer=True)
    g, meta, net, _ = run_grads(dl, name)
    check_against_golden(g, meta, net)


def test_grads_deterministic(dl):
    a = run_grads(dl, "grad_v4_med")[2]
    b = run_grads(dl, "grad_v4_med")[2]
    for (ka, pa), (kb, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(pa.grad, pb.grad), ka


@pytest.mark.parametrize("variant", ["v4", "v2"])
def test_grads_match_oracle_larger_batch(variant, dl):
    """B = 333 (ragged, 6 column tiles) at m=250, n=500 against the backward oracle."""
    from oracle import dladmm_oracle as fwd
    from oracle import dladmm_oracle_grad as og
    m, n, B, K = 250, 500, 333, 4
    d = dict(variant=variant, m=m, n=n, B=B, K=K, seed=9100, perturb=0.1, wscale=0.4)
    inp, sd = P.build_problem(d)
    up = P.make_upstream(d, P.VARIANT_SPECS[variant]["ret_t"])
    net = make_train_net(dl, variant, inp, sd, K)
    X = torch.from_numpy(inp["X"]).cuda()
    A = torch.from_numpy(inp["A"]).cuda()
    loss = total_loss(net(X), X, A, up, "l1l1", K)
    loss.backward()
    ref = {}
    for dt in (np.float32, np.float64):
        o = fwd.forward(variant, inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, K,
                        dtype=dt)
        gz = og.train_loss_grads(o["Z"], inp["X"], inp["A"], P.GRAD_ALPHA, P.loss_coeffs(K),
                                 "l1l1", dtype=dt)
        gz = [a + b for a, b in zip(gz, up["Gz"])]
        ref[dt] = og.vjp(variant, inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, K,
                         gZ=gz, gE=list(up["Ge"]), gL=list(up["Gl"]),
                         gT=list(up["Gt"]) if "Gt" in up else None, dtype=dt)
    for key, p in net.named_parameters():
        # against the fp64 oracle, within the fp32 oracle's own distance from it
        gap = nrel(ref[np.float32][key], ref[np.float64][key])
        e = nrel(p.grad.cpu().numpy(), ref[np.float64][key])
        assert e <= max(GTOL, 3.0 * gap), (key, e, gap)


def test_adam_training_step(dl):
    """One reference training step (main_syn_l1l1_scalar.py:269-299: zero_grad, forward, loss,
    backward, Adam step) moves the parameters exactly as the same step driven by the oracle's
    gradients."""
    name = "grad_v4_small"
    g, meta = load_golden(name)
    d = meta["defn"]
    inp, sd = P.build_problem(d)
    up = P.make_upstream(d, True)
    net = make_train_net(dl, "v4", inp, sd, d["K"])
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    opt.zero_grad()
    X = torch.from_numpy(inp["X"]).cuda()
    A = torch.from_numpy(inp["A"]).cuda()
    total_loss(net(X), X, A, up, "l1l1", d["K"]).backward()
    opt.step()
    # the same Adam step on CPU parameters whose .grad is the reference autograd gradient
    ref = {k: torch.nn.Parameter(torch.from_numpy(v.copy())) for k, v in sd.items()}
    opt2 = torch.optim.Adam(list(ref.values()), lr=1e-3)
    for k, p in ref.items():
        p.grad = torch.from_numpy(g["g:" + k])
    opt2.step()
    for k, p in net.named_parameters():
        np.testing.assert_allclose(p.detach().cpu().numpy(), ref[k].detach().numpy(),
                                   rtol=0, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("name,precision", grad_cases(
    ["grad_v4_med", "grad_v6_med", "grad_v1_small", "grad_v2_ragged", "grad_v5_small",
     "grad_v3_small"]))
def test_fused_training_loss(name, precision, dl, monkeypatch):
    """net.training_loss (objective reduced in the forward kernel, its gradient injected in the
    backward kernels) == the reference loss built from the outputs with torch ops: same value,
    same gradients (against the oracle's reverse sweep of the same loss and against reference
    autograd through the module's outputs), at both training precisions."""
    from oracle import dladmm_oracle as fwd
    from oracle import dladmm_oracle_grad as og
    g, meta = load_golden(name)
    d = meta["defn"]
    kind = meta["gdef"]["loss"]
    K = d["K"]
    inp, sd = P.build_problem(d)
    X = torch.from_numpy(inp["X"]).cuda()
    A = torch.from_numpy(inp["A"]).cuda()
    coeffs = P.loss_coeffs(K)
    paths = record_paths(monkeypatch)
    net = make_train_net(dl, d["variant"], inp, sd, K, precision=precision, **P.ctor_extra(d))
    total, per_layer = net.training_loss(X, P.GRAD_ALPHA, coeffs, kind)
    total.backward()
    if precision == "f32_split":
        assert paths[0] == (4 if split_expected(d) else 1), paths
    net2 = make_train_net(dl, d["variant"], inp, sd, K, **P.ctor_extra(d))
    ref_total = total_loss(net2(X), X, A, {"Gz": np.zeros((K, 1, 1), np.float32),
                                          "Ge": np.zeros((K, 1, 1), np.float32),
                                          "Gl": np.zeros((K, 1, 1), np.float32)}, kind, K)
    ref_total.backward()
    np.testing.assert_allclose(float(total), float(ref_total), rtol=1e-5)
    assert per_layer.shape == (K,)
    res = {}
    for dt in (np.float32, np.float64):
        o = fwd.forward(d["variant"], inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, K,
                        dtype=dt)
        gz = og.train_loss_grads(o["Z"], inp["X"], inp["A"], P.GRAD_ALPHA, coeffs, kind, dtype=dt)
        res[dt] = og.vjp(d["variant"], inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd,
                         K, gZ=gz, dtype=dt)
    p2 = dict(net2.named_parameters())
    for key, p in net.named_parameters():
        # the objective reads Z only: the last layer's E/L-step parameters are outside the
        # graph, so reference autograd leaves their .grad None (the oracle's VJP is 0 there)
        assert (p.grad is None) == (key in none_keys(name, "training_loss")), key
        if p.grad is None:
            # net2's loss adds 0 * E_k, 0 * L_k terms, which put them in the graph (zero grads)
            assert p2[key].grad is None or not torch.any(p2[key].grad), key
            assert not np.any(res[np.float64][key]), key
            continue
        gap = nrel(res[np.float32][key], res[np.float64][key])
        e = nrel(p.grad.cpu().numpy(), res[np.float64][key])
        parity.check(name + " fused objective grad vs oracle64", precision, key, e,
                     max(GTOL, 3.0 * gap), gap)
        e2 = nrel(p.grad.cpu().numpy(), p2[key].grad.cpu().numpy())
        parity.check(name + " fused objective grad vs torch-op loss", precision, key, e2,
                     max(GTOL, 3.0 * gap), gap)


@pytest.mark.parametrize("variant", ["v4", "v1", "v2", "v3", "v5", "v6"])
@pytest.mark.parametrize("lossy", [False, True])
def test_saved_product_backward(variant, lossy, dl, flags):
    """A training forward on the fused kernel keeps P_k = A Z_k (fwd_desc.P) and BK1 reads it
    instead of recomputing the product, inside BK3's launch (phase 6).
      (a) phase 6 == BK1 as its own launch (flags bwd_unfused): every elementwise adjoint,
          the weight and the per-sample gradients bit for bit, the parameter-slot sums to their
          fp32 partials' rounding (the partials group the terms by wave differently);
      (b) the saved P is A Z_k of the returned Z_k, and storing it changes no other output;
      (c) a backward that recomputes P with the slice GEMM (a forward without P) agrees to fp32
          rounding: the fused forward sums A Z_k in two accumulation chains, the slice GEMM in
          one, so the recomputed P differs in the last bits."""
    from importlib import import_module
    ops = import_module("d-ladmm_amd.ops")
    m, n, B, K = 96, 200, 70, 4
    d = dict(variant=variant, m=m, n=n, B=B, K=K, seed=9500, perturb=0.1,
             wscale=0.4 if variant in ("v1", "v2") else None)
    inp, sd = P.build_problem(d)
    net = make_train_net(dl, variant, inp, sd, K)
    net.cuda()
    X = torch.from_numpy(inp["X"]).cuda()
    with torch.no_grad():
        tables = net._tables(X.device)
    W = [w.detach() for w in net._weights()]
    lk = dl._lib.LOSS_LASSO if variant == "v6" else dl._lib.LOSS_L1L1
    args = (net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0)
    with torch.no_grad():
        r1 = ops.dladmm_forward(*args, keep_all=True, want_T=True, want_P=True,
                                loss_kind=lk if lossy else 0, **tables)
        r0 = ops.dladmm_forward(*args, keep_all=True, want_T=True,
                                loss_kind=lk if lossy else 0, **tables)
    assert r1.P is not None and r0.P is None
    for a, b in ((r1.Z, r0.Z), (r1.E, r0.E), (r1.L, r0.L), (r1.T, r0.T)):
        assert torch.equal(a, b)  # the extra store changes nothing else
    Pref = torch.einsum("mn,knb->kmb", net.A.double(), r1.Z.double())
    assert float((r1.P.double() - Pref).norm() / Pref.norm()) < 1e-6
    g = torch.Generator(device="cuda").manual_seed(5)
    gz = [torch.randn(n, B, device="cuda", generator=g) for _ in range(K)]
    ge = [torch.randn(m, B, device="cuda", generator=g) for _ in range(K)]
    gl = [torch.randn(m, B, device="cuda", generator=g) for _ in range(K)]
    gt = [torch.randn(m, B, device="cuda", generator=g) for _ in range(K + 1)]
    kw = dict(tied=net._shared_weight(), **tables)
    if lossy:
        kw.update(loss_kind=lk, loss_coef=torch.tensor([[1e-3, 1.0]] * K, device="cuda"))
    fused = ops.dladmm_backward(*args, r1, gz, ge, gl, gt, **kw)
    flags.set(bwd_unfused=True)
    unfused = ops.dladmm_backward(*args, r1, gz, ge, gl, gt, **kw)
    flags.set(bwd_unfused=False)
    recomp = ops.dladmm_backward(*args, r0, gz, ge, gl, gt, **kw)
    for other, exact in ((unfused, True), (recomp, False)):
        for f in ("gW", "g_scalar", "g_row"):
            a, b = getattr(fused, f), getattr(other, f)
            assert (a is None) == (b is None)
            if a is None:
                continue
            if f == "gW" and exact:
                assert torch.equal(a, b), f
            else:
                assert nrel(a.cpu().numpy(), b.cpu().numpy()) <= (2e-6 if exact else 1e-4), f
        for a, b in zip(fused.g_beta1 + fused.g_beta2, other.g_beta1 + other.g_beta2):
            if exact:
                assert torch.equal(a, b)
            else:
                assert nrel(a.cpu().numpy(), b.cpu().numpy()) <= 1e-4
