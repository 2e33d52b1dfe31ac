"""Parity of the fused HIP forward (through the C ABI) with the reference.

* golden fixtures (outputs of the reference classes, tests/golden/) -- every variant, every layer;
* the oracle (CPU restatement pinned by those fixtures) at larger / ragged batches;
* size-independent properties at the BASELINE shape (columns are independent samples, so any
  column subset must match the oracle run on just those columns; the fused per-layer objective
  must equal a separate reduction of the returned outputs; runs are bitwise deterministic).

Tolerance (tests/parity.py: north_star + BASELINE.md "Parity"), per layer, norm-relative: within
1e-5 of the reference's fp32 output, or -- where the reference's own fp32 rounding puts that out of
reach (the ill-conditioned V1 default init) -- at most 2 x as far from the exact (fp64) result as
the reference's fp32 output is.  Every checked error is recorded (DLADMM_PARITY_JSON).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
import parity
import problems as P

pytestmark = pytest.mark.gpu

REL = parity.REL
nrel = parity.nrel


def _path_name(net):
    return {"f32": "f32", "f32_split": "split", "bf16": "bf16"}[net.precision]


def make_net(dl, variant, inp, sd, K, **extra):
    m, n = inp["A"].shape
    B = inp["X"].shape[1]
    cls = dl.VARIANTS[variant]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    net = cls(m=m, n=0, d=n, batch_size=B, A=t(inp["A"]), Z0=t(inp["Z0"]), E0=t(inp["E0"]),
              L0=t(inp["L0"]), layers=K, **extra)
    net.load_state_dict({k: t(v) for k, v in sd.items()}, strict=True)
    net.requires_grad_(False)
    return net


@pytest.mark.parametrize("name", sorted(P.FIXTURES))
def test_matches_reference_golden(name, dl):
    g, meta = load_golden(name)
    d = meta["defn"]
    inp, sd = P.build_problem(d)
    net = make_net(dl, d["variant"], inp, sd, d["K"], **P.ctor_extra(d))
    X = torch.from_numpy(inp["X"]).cuda()
    with torch.no_grad():
        out = net(X)
    torch.cuda.synchronize()
    assert len(out) == (4 if "T" in g.files else 3)
    check_golden(name, g, meta, net, X, out)


@pytest.mark.parametrize("name", sorted(P.FIXTURES))
def test_per_layer_path_matches_reference_golden(name, dl, flags):
    """The same fixtures through the per-layer kernel pairs (flags per_layer: the path of
    every shape beyond the fused kernel's, e.g. BASELINE config 4)."""
    g, meta = load_golden(name)
    d = meta["defn"]
    inp, sd = P.build_problem(d)
    net = make_net(dl, d["variant"], inp, sd, d["K"], **P.ctor_extra(d))
    X = torch.from_numpy(inp["X"]).cuda()
    flags.set(per_layer=True)
    with torch.no_grad():
        out = net(X)
    check_golden(name, g, meta, net, X, out, path="layered")


_R64 = {}


def _golden_r64(name, meta):
    """The oracle's fp64 forward of a golden fixture (the exact result the gap is measured to)
    and its fp32 forward (the second CPU fp32 evaluation of the reference algorithm)."""
    if name not in _R64:
        from oracle import dladmm_oracle as O
        d = meta["defn"]
        inp, sd = P.build_problem(d)
        args = (d["variant"], inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, d["K"])
        _R64[name] = (O.forward(*args, dtype=np.float64), O.forward(*args))
    return _R64[name]


def check_golden(name, g, meta, net, X, out, path=None):
    """Every layer's outputs against the reference's golden fp32 outputs (and the exact fp64
    result), and the fused per-layer objectives against the reference training loop's loss
    values, at the parity bar."""
    path = path or _path_name(net)
    names = ["Z", "E", "L", "T"][: len(out)]
    r64, o32 = _golden_r64(meta["name"], meta)
    for nm, seq in zip(names, out):
        ref = g[nm]
        assert len(seq) == ref.shape[0]
        for k, t in enumerate(seq):
            # the reference algorithm's fp32 error: the reference's own (torch) run and the
            # numpy restatement's, the larger (tests/parity.py)
            gap = max(float(g["gap_" + nm][k]), nrel(o32[nm][k], r64[nm][k]))
            got = t.cpu().numpy()
            parity.check_f32(name, path, f"{nm}[{k}]", nrel(got, ref[k]), nrel(got, r64[nm][k]),
                             gap)
    # fused per-layer objective (the training loop's loss[k]); its bar follows the conditioning
    # of the layer outputs it is computed from
    gmax = max(float(np.max(g["gap_" + nm])) for nm in names)
    for kind in ("l1l1", "lasso"):
        _, obj = net.layer_objectives(X, meta["alpha"], kind)
        ref = g["loss_" + kind]
        err = float(np.max(np.abs(obj.cpu().numpy() - ref) / np.abs(ref)))
        parity.check(name, path, f"objective {kind}", err, parity.tol(gmax), gmax)


def _oracle_case(oracle, variant, m, n, B, K, seed, perturb=0.1, wscale=None, sd=None):
    inp = P.make_inputs(m, n, B, seed)
    if sd is None:
        sd = P.make_state_dict(variant, m, n, B, K, inp["A"], seed, perturb=perturb,
                               wscale=wscale)
    r32, ref64, gap, ref = parity.fp32_refs(oracle, variant, inp["X"], inp["A"], inp["Z0"],
                                            inp["E0"], inp["L0"], sd, K)
    ref.update(r32)   # ref32 = the reference's own op sequence (torch restatement)
    ref["Xs"] = inp["X"]
    ref["gap"] = gap
    ref["r64"] = ref64
    return inp, sd, ref


def _compare(out, ref, tag="", path="f32"):
    """Per layer, against the fp64 oracle: nrel(gpu, oracle64) <= max(1e-5, 2 x nrel(oracle32,
    oracle64)) -- the GPU's fp32 result may be as far from the exact one as the reference's own
    fp32 evaluation is (it sums its GEMMs in another order).  Every output is measured by its own
    norm, T (= A Z + E - X, a small residual) included: where that residual's rounding puts 1e-5
    out of reach, the gap clause applies."""
    names = ["Z", "E", "L", "T"][: len(out)]
    for nm, seq in zip(names, out):
        for k, t in enumerate(seq):
            r = np.asarray(ref["r64"][nm][k], np.float64)
            r32 = np.asarray(ref[nm][k], np.float64)
            got = t.cpu().numpy().astype(np.float64)
            e32, e64, gap = nrel(got, r32), nrel(got, r), ref["gap"][nm][k]
            parity.check_f32(tag, path, f"{nm}[{k}] vs oracle", e32, e64, gap)


@pytest.mark.parametrize("variant", ["v1", "v2", "v3", "v4", "v5", "v6"])
@pytest.mark.parametrize("B", [1, 64, 300])
def test_variants_vs_oracle_baseline_shape(variant, B, dl, oracle):
    """m=256, n=512, K=15 (BASELINE shape), ragged / tiny batches, perturbed params."""
    m, n, K = 256, 512, 15
    inp, sd, ref = _oracle_case(oracle, variant, m, n, B, K, seed=2000 + B,
                                wscale=0.4 if variant in ("v1", "v2") else None)
    net = make_net(dl, variant, inp, sd, K)
    with torch.no_grad():
        out = net(torch.from_numpy(inp["X"]).cuda())
    _compare(out, ref, tag=f"{variant} B={B}")


@pytest.mark.parametrize("shape", [(16, 32), (30, 70), (64, 256), (250, 500), (200, 512)])
def test_padded_shapes_vs_oracle(shape, dl, oracle):
    """Shapes that are not the instantiation's size run zero-padded; padding must be exact."""
    m, n = shape
    for variant in ("v4", "v2", "v1"):
        inp, sd, ref = _oracle_case(oracle, variant, m, n, 77, 5, seed=3000 + m,
                                    wscale=0.4 if variant in ("v1", "v2") else None)
        net = make_net(dl, variant, inp, sd, 5)
        with torch.no_grad():
            out = net(torch.from_numpy(inp["X"]).cuda())
        _compare(out, ref, tag=f"{variant} {shape}")


def test_single_layer_and_negative_thresholds(dl, oracle):
    m, n, B = 256, 512, 100
    inp = P.make_inputs(m, n, B, 4001)
    sd = P.make_state_dict("v4", m, n, B, 1, inp["A"], 4001, perturb=0.2)
    sd["active_para.0"][:] = -0.05  # literal two-relu shrink with theta < 0
    inp, sd, ref = _oracle_case(oracle, "v4", m, n, B, 1, 4001, sd=sd)
    net = make_net(dl, "v4", inp, sd, 1)
    with torch.no_grad():
        out = net(torch.from_numpy(inp["X"]).cuda())
    _compare(out, ref, tag="K=1 negtheta")


def test_lean_mode_and_determinism(dl):
    """keep_all=False writes only the last layer: bit-identical to the full run's last layer;
    two runs are bitwise identical (no atomics, fixed reduction order)."""
    m, n, B, K = 256, 512, 1000, 15
    inp = P.make_inputs(m, n, B, 5001)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 5001, perturb=0.1)
    net = make_net(dl, "v4", inp, sd, K)
    X = torch.from_numpy(inp["X"]).cuda()
    with torch.no_grad():
        full = net.run(X, keep_all=True, loss_kind=1)
        full2 = net.run(X, keep_all=True, loss_kind=1)
        lean = net.run(X, keep_all=False, loss_kind=1)
    for a, b in ((full.Z, full2.Z), (full.E, full2.E), (full.L, full2.L), (full.T, full2.T),
                 (full.loss_sums, full2.loss_sums)):
        assert torch.equal(a, b)
    assert torch.equal(lean.Z[0], full.Z[-1])
    assert torch.equal(lean.E[0], full.E[-1])
    assert torch.equal(lean.L[0], full.L[-1])
    assert torch.equal(lean.T[0], full.T[-1])
    assert torch.equal(lean.loss_sums, full.loss_sums)


def test_strided_batch_views(dl, oracle):
    """Inputs/outputs addressed through leading dimensions: a column slice of a wider X
    (what a batch shard of a larger array looks like) gives the same result."""
    m, n, B, K = 256, 512, 200, 4
    inp = P.make_inputs(m, n, 3 * B, 6001)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 6001, perturb=0.1)
    Xw = torch.from_numpy(inp["X"]).cuda()
    Xv = Xw[:, B:2 * B]
    assert Xv.stride(0) == 3 * B
    net = make_net(dl, "v4", dict(inp, X=inp["X"][:, B:2 * B], Z0=inp["Z0"][:, B:2 * B],
                                  E0=inp["E0"][:, B:2 * B], L0=inp["L0"][:, B:2 * B]), sd, K)
    with torch.no_grad():
        out_v = net(Xv)
        out_c = net(Xv.contiguous())
    for a, b in zip(out_v, out_c):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


def test_errors_are_loud(dl):
    m, n, B, K = 16, 32, 8, 2
    inp = P.make_inputs(m, n, B, 7001)
    sd = P.make_state_dict("v1", m, n, B, K, inp["A"], 7001)
    net = make_net(dl, "v1", inp, sd, K)
    with torch.no_grad():
        with pytest.raises(RuntimeError):   # V1 betas are (m, batch_size): B must match
            net(torch.zeros(m, B + 1, device="cuda"))
        with pytest.raises(RuntimeError):   # no CPU fallback
            net(torch.zeros(m, B))
    net.requires_grad_(True)
    with pytest.raises(RuntimeError):       # no gradients w.r.t. the input X (reference: data)
        net(torch.zeros(m, B, device="cuda", requires_grad=True))


def test_baseline_size_column_subset_and_fused_loss(dl, oracle):
    """B = 65,536 (north-star shape).  Columns are independent, so the oracle on a random subset
    of columns must reproduce those columns; the fused loss must equal a separate reduction."""
    m, n, K, B = 256, 512, 15, 65536
    g = torch.Generator(device="cpu").manual_seed(8001)
    inp = P.make_inputs(m, n, 64, 8001)            # A and a template; X regenerated below
    A = inp["A"]
    rng = np.random.default_rng(8002)
    zs = (rng.random((n, B)) < 0.1) * rng.standard_normal((n, B))
    es = (rng.random((m, B)) < 0.1) * rng.standard_normal((m, B))
    X = (A.astype(np.float64) @ zs + es).astype(np.float32)
    Z0 = (rng.random((n, B)) / n).astype(np.float32)
    E0 = np.zeros((m, B), np.float32)
    L0 = np.zeros((m, B), np.float32)
    sd = P.make_state_dict("v4", m, n, B, K, A, 8001, perturb=0.1)
    full = dict(A=A, X=X, Z0=Z0, E0=E0, L0=L0)
    net = make_net(dl, "v4", full, sd, K)
    Xd = torch.from_numpy(X).cuda()
    with torch.no_grad():
        r, obj = net.layer_objectives(Xd, 0.001, "l1l1")
    torch.cuda.synchronize()
    cols = np.sort(torch.randperm(B, generator=g)[:96].numpy())
    ref = oracle.forward("v4", X[:, cols], A, Z0[:, cols], E0[:, cols], L0[:, cols], sd, K)
    for nm, got in (("Z", r.Z), ("E", r.E), ("L", r.L)):
        for k in range(K):
            e = nrel(got[k][:, cols].cpu().numpy(), ref[nm][k])
            parity.check("v4 B=65536 columns", "f32", f"{nm}[{k}] vs oracle32", e, REL)
    # fused objective == separate reduction of the returned outputs (fp64 on device)
    Ad = torch.from_numpy(A).cuda().double()
    sep = []
    for k in range(K):
        Zk = r.Z[k].double()
        sep.append(float((0.001 * Zk.abs().sum() + (Xd.double() - Ad @ Zk).abs().sum()) / B))
    np.testing.assert_allclose(obj.cpu().numpy(), np.array(sep), rtol=1e-5)


# ------------------------------------------------------------------ per-layer path (path 2)
@pytest.mark.parametrize("variant", ["v1", "v2", "v3", "v4", "v5", "v6"])
def test_per_layer_path_vs_oracle(variant, dl, oracle):
    """m > 256: beyond the fused kernel's register budget -> per-layer kernel pairs."""
    m, n, B, K = 300, 600, 150, 6
    inp, sd, ref = _oracle_case(oracle, variant, m, n, B, K, seed=9000 + K,
                                wscale=0.4 if variant in ("v1", "v2") else None)
    net = make_net(dl, variant, inp, sd, K)
    with torch.no_grad():
        out = net(torch.from_numpy(inp["X"]).cuda())
    _compare(out, ref, tag=f"layered {variant}", path="layered")


@pytest.mark.parametrize("variant", ["v4", "v1", "v6"])
def test_forced_per_layer_path_matches_fused(variant, dl, flags):
    """The same problem through both paths (flags per_layer forces path 2): outputs agree
    to fp32 summation-order noise, the lean mode and the fused objective too."""
    m, n, B, K = 256, 512, 333, 5
    inp = P.make_inputs(m, n, B, 9100)
    sd = P.make_state_dict(variant, m, n, B, K, inp["A"], 9100, perturb=0.1, wscale=0.4)
    net = make_net(dl, variant, inp, sd, K)
    X = torch.from_numpy(inp["X"]).cuda()
    with torch.no_grad():
        rf, of = net.layer_objectives(X, 0.001, "l1l1")
        flags.set(per_layer=True)
        rl, ol = net.layer_objectives(X, 0.001, "l1l1")
        lean = net.run(X, keep_all=False)
        flags.set(per_layer=False)
    for a, b in ((rf.Z, rl.Z), (rf.E, rl.E), (rf.L, rl.L)):
        for k in range(K):
            assert nrel(b[k].cpu().numpy(), a[k].cpu().numpy()) <= 2e-6
    assert torch.equal(lean.Z[0], rl.Z[-1]) and torch.equal(lean.L[0], rl.L[-1])
    np.testing.assert_allclose(ol.cpu().numpy(), of.cpu().numpy(), rtol=2e-6)


@pytest.mark.parametrize("variant,extra", [("v7", {}), ("v7t", {}), ("v7p", {"interval": 2})])
def test_news_partial_depth(variant, extra, dl, oracle):
    """newS forward(x, K) runs min(K, layers) layers (main_syn_scalar_newS_layerwise.py:78)."""
    d = dict(variant=variant, m=64, n=256, B=40, K=6, seed=7301, perturb=0.2, **extra)
    inp, sd = P.build_problem(d)
    net = make_net(dl, variant, inp, sd, 6, **extra)
    X = torch.from_numpy(inp["X"]).cuda()
    for K in (1, 4, 9):
        nl = min(K, 6)
        with torch.no_grad():
            Z, E, L = net(X, K)
        assert len(Z) == len(E) == len(L) == nl
        ref = oracle.forward(variant, inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, nl)
        r64 = oracle.forward(variant, inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, nl,
                             dtype=np.float64)
        for nm, seq in (("Z", Z), ("E", E), ("L", L)):
            for k in range(nl):
                got = seq[k].cpu().numpy()
                parity.check_f32(f"{variant} newS K={K}", "f32", f"{nm}[{k}] vs oracle",
                                 nrel(got, ref[nm][k]), nrel(got, r64[nm][k]),
                                 nrel(ref[nm][k], r64[nm][k]))


@pytest.mark.parametrize("precision", ["f32", "bf16"])
def test_strided_views_per_layer_paths(precision, dl):
    """Per-layer (m > 256) and bf16-tile paths with every input a column slice of a wider array
    (odd leading dimension 3B, B = 201): the state DMAs and epilogues address through ld, so the
    result equals the contiguous run bit for bit."""
    m, n, B, K = 300, 530, 201, 3
    inp = P.make_inputs(m, n, 3 * B, 6002)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 6002, perturb=0.1)
    sl = slice(B, 2 * B)
    net = make_net(dl, "v4", dict(inp, X=inp["X"][:, sl], Z0=inp["Z0"][:, sl],
                                  E0=inp["E0"][:, sl], L0=inp["L0"][:, sl]), sd, K)
    net.precision = precision
    Xw = torch.from_numpy(inp["X"]).cuda()
    Xv = Xw[:, sl]
    assert Xv.stride(0) == 3 * B
    with torch.no_grad():
        out_v = net(Xv)
        out_c = net(Xv.contiguous())
    for a, b in zip(out_v, out_c):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


@pytest.mark.parametrize("variant", ["v1", "v4", "v6"])
def test_empty_batch(variant, dl, oracle):
    """batch_size = 0: the reference's ops return K empty (rows, 0) tensors (and T), so does the
    drop-in (no kernel runs); the fused objective sums are zero and a training step leaves zero
    gradients."""
    m, n, K = 24, 40, 3
    inp = P.make_inputs(m, n, 0, 3)
    sd = P.make_state_dict(variant, m, n, 0, K, inp["A"], 3)
    t = torch.from_numpy
    net = dl.VARIANTS[variant](m=m, n=0, d=n, batch_size=0, A=t(inp["A"]), Z0=t(inp["Z0"]),
                               E0=t(inp["E0"]), L0=t(inp["L0"]), layers=K)
    net.load_state_dict({k: t(v) for k, v in sd.items()})
    ref = oracle.forward(variant, inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, K)
    X = t(inp["X"]).cuda()
    with torch.no_grad():
        out = net(X)
    assert len(out) == (4 if variant != "v1" else 3)
    for i, nm in enumerate("ZELT"[:len(out)]):
        assert len(out[i]) == len(ref[nm])
        for a, b in zip(out[i], ref[nm]):
            assert tuple(a.shape) == b.shape
    with torch.no_grad():
        r = net.run(X, keep_all=True, loss_kind=1)
    assert torch.count_nonzero(r.loss_sums) == 0
    if variant == "v4":
        net.requires_grad_(True)
        total, _ = net.training_loss(X, 0.001, [1.0] * K, "l1l1")
        total.backward()
        for p in net.parameters():
            assert p.grad is None or torch.count_nonzero(p.grad) == 0


@pytest.mark.parametrize("layered", [False, True])
def test_v1_deeper_than_64_layers(layered, dl, oracle, flags):
    """The reference V1 ctor has no depth limit (main_lena.py:30-41): the fused kernel reads the
    per-layer beta pointers from a device table, so K = 80 runs (both paths)."""
    m, n, B, K = 16, 32, 24, 80
    inp, sd, ref = _oracle_case(oracle, "v1", m, n, B, K, seed=9400, wscale=0.4)
    net = make_net(dl, "v1", inp, sd, K)
    if layered:
        flags.set(per_layer=True)
    with torch.no_grad():
        out = net(torch.from_numpy(inp["X"]).cuda())
    assert len(out[0]) == K
    _compare(out, ref, tag=f"v1 K={K}", path="layered" if layered else "f32")
