"""BASELINE config 5: bf16 MFMA operands with fp32 accumulation and an fp32 dual / state
(precision="bf16", per-layer kernel path 3).

Tolerance re-stated for this mode (north_star: "tolerance re-stated").  Let s_k be the distance
(norm-relative, per layer) that bf16 operand rounding itself puts between the oracle's bf16
restatement (oracle.forward(gemm="bf16"): operands rounded to bf16 RNE, products accumulated
exactly, elementwise fp32) and the fp32 reference.  The GPU result must be within 0.25 s_k of the
bf16 restatement (it tracks the bf16 algorithm, not just "something near fp32") and within
1.25 s_k of the fp32 reference.  The slack covers the fp32 MFMA accumulation order and the
state elements whose bf16 rounding falls on the other side of a rounding boundary when the
fp32 state differs in its last bits.

Where the iteration amplifies rounding (the config-5 shape m=1024, n=4096 at depth 15: s_k grows
to 0.11), those boundary flips compound: two valid bf16 implementations that differ only in the
accumulation order drift apart by d_k (~0.3 s_k by layer 15; measured on the reference itself,
tests/golden/make_golden_bf16.py).  `bf16_bar` therefore allows max(0.25 s_k, 2 d_k) from the bf16
reference and s_k + that from the fp32 reference (the triangle inequality); on the small shapes
d_k ~ 0 and the bar is the 0.25 / 1.25 s_k one.
"""
import numpy as np
import pytest
import torch

import problems as P

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["wide", "narrow"])
def tile(request, flags):
    """Every test runs on both tile widths (256 columns / 8 waves, 128 columns / 4 waves with
    two workgroups per CU; plan flag bf16_wide, i.e. DLADMM_F_BF16_WIDE in the descriptor)."""
    flags.set(bf16_wide=request.param == "wide")
    return request.param


def bf16_bar(s, d):
    """(bound vs the bf16 reference, bound vs the fp32 reference) for yardsticks s_k, d_k."""
    b = max(1e-5, 0.25 * s, 2.0 * d)
    return b, 1e-5 + max(1.25 * s, s + b)


def nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def run(dl, variant, m, n, B, K, seed):
    d = dict(variant=variant, m=m, n=n, B=B, K=K, seed=seed, perturb=0.1,
             wscale=0.4 if variant in ("v1", "v2") else None)
    inp, sd = P.build_problem(d)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    net = dl.VARIANTS[variant](m=m, n=0, d=n, batch_size=B, A=t(inp["A"]), Z0=t(inp["Z0"]),
                               E0=t(inp["E0"]), L0=t(inp["L0"]), layers=K)
    net.load_state_dict({k: t(v) for k, v in sd.items()})
    net.requires_grad_(False)
    net.precision = "bf16"
    with torch.no_grad():
        out = net(t(inp["X"]).cuda())
    return inp, sd, out


@pytest.mark.parametrize("variant", ["v4", "v6", "v1", "v3", "v5"])
def test_bf16_tracks_bf16_restatement(variant, dl, oracle):
    m, n, B, K = 96, 200, 70, 6
    inp, sd, out = run(dl, variant, m, n, B, K, 9300)
    args = (variant, inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, K)
    rb = oracle.forward(*args, gemm="bf16")
    r32 = oracle.forward(*args)
    for i, nm in enumerate("ZEL"):
        for k in range(K):
            got = out[i][k].cpu().numpy()
            scale = nrel(rb[nm][k], r32[nm][k])        # what bf16 rounding costs
            assert nrel(got, rb[nm][k]) <= max(1e-5, 0.25 * scale), (nm, k)
            assert nrel(got, r32[nm][k]) <= 1e-5 + 1.25 * scale, (nm, k)


def test_bf16_config5_shape(dl, oracle):
    """m = 1024, n = 4096 (config 5) at a column slice, 3 layers."""
    m, n, B, K = 1024, 4096, 64, 3
    inp, sd, out = run(dl, "v4", m, n, B, K, 9301)
    args = ("v4", inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, K)
    rb = oracle.forward(*args, gemm="bf16")
    r32 = oracle.forward(*args)
    for i, nm in enumerate("ZELT"):
        for k in range(K):
            got = out[i][k].cpu().numpy()
            scale = nrel(rb[nm][k], r32[nm][k])
            assert nrel(got, rb[nm][k]) <= max(1e-5, 0.25 * scale), (nm, k)
            assert nrel(got, r32[nm][k]) <= 1e-5 + 1.25 * scale, (nm, k)


def test_bf16_is_inference_only(dl):
    inp = P.make_inputs(16, 32, 4, 1)
    t = torch.from_numpy
    net = dl.DLADMMNetScalar(m=16, n=0, d=32, batch_size=4, A=t(inp["A"]), Z0=t(inp["Z0"]),
                             E0=t(inp["E0"]), L0=t(inp["L0"]), layers=2)
    net.precision = "bf16"
    with pytest.raises(RuntimeError):
        net(t(inp["X"]).cuda())


@pytest.mark.parametrize("variant", ["v4", "v2", "v6"])
def test_bf16_multi_tile_ragged(variant, dl, oracle):
    """Several 256 x 256 tiles in both directions with ragged edges (rows m, n and batch B not
    multiples of 16 / 32 / 256): the packed-state padding and the per-tile epilogue offsets."""
    m, n, B, K = 300, 530, 600, 3
    inp, sd, out = run(dl, variant, m, n, B, K, 9302)
    args = (variant, inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, K)
    rb = oracle.forward(*args, gemm="bf16")
    r32 = oracle.forward(*args)
    for i, nm in enumerate("ZEL"):
        for k in range(K):
            got = out[i][k].cpu().numpy()
            scale = nrel(rb[nm][k], r32[nm][k])
            assert nrel(got, rb[nm][k]) <= max(1e-5, 0.25 * scale), (variant, nm, k)
            assert nrel(got, r32[nm][k]) <= 1e-5 + 1.25 * scale, (variant, nm, k)


def test_bf16_loss_lean_and_determinism(dl):
    """Fused per-layer objective sums equal the objective recomputed from the returned Z/E/T
    (fp64, 1e-6 relative: the sums are fp32 partials reduced in fixed order); lean mode returns
    the full run's last layer bit for bit; two runs are bitwise identical."""
    m, n, B, K = 288, 544, 520, 4
    inp = P.make_inputs(m, n, B, 9303)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 9303, perturb=0.1)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    net = dl.VARIANTS["v4"](m=m, n=0, d=n, batch_size=B, A=t(inp["A"]), Z0=t(inp["Z0"]),
                            E0=t(inp["E0"]), L0=t(inp["L0"]), layers=K)
    net.load_state_dict({k: t(v) for k, v in sd.items()})
    net.requires_grad_(False)
    net.cuda()
    net.precision = "bf16"
    X = t(inp["X"]).cuda()
    with torch.no_grad():
        full = net.run(X, keep_all=True, loss_kind=1)
        full2 = net.run(X, keep_all=True, loss_kind=1)
        lean = net.run(X, keep_all=False, loss_kind=1)
    for a, b in ((full.Z, full2.Z), (full.E, full2.E), (full.L, full2.L), (full.T, full2.T),
                 (full.loss_sums, full2.loss_sums)):
        assert torch.equal(a, b)
    for a, b in ((lean.Z[0], full.Z[-1]), (lean.E[0], full.E[-1]), (lean.L[0], full.L[-1]),
                 (lean.T[0], full.T[-1]), (lean.loss_sums, full.loss_sums)):
        assert torch.equal(a, b)
    ls = full.loss_sums.cpu().numpy()
    for k in range(K):
        z = full.Z[k].double().cpu().numpy()
        res = (full.E[k] - full.T[k + 1]).double().cpu().numpy()   # X - A Z_k = E_k - T_{k+1}
        assert abs(ls[k, 0] - np.abs(z).sum()) <= 1e-6 * np.abs(z).sum(), k
        assert abs(ls[k, 1] - np.abs(res).sum()) <= 1e-4 * np.abs(res).sum(), k


def test_bf16_tile_widths_bit_identical(dl, flags):
    """Both tile widths compute every output element as the same chain (k-blocks in order, same
    packed operands, same epilogue code): the outputs and fused sums are bitwise equal."""
    m, n, B, K = 300, 530, 600, 3
    inp = P.make_inputs(m, n, B, 9304)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 9304, perturb=0.1)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    net = dl.VARIANTS["v4"](m=m, n=0, d=n, batch_size=B, A=t(inp["A"]), Z0=t(inp["Z0"]),
                            E0=t(inp["E0"]), L0=t(inp["L0"]), layers=K)
    net.load_state_dict({k: t(v) for k, v in sd.items()})
    net.requires_grad_(False)
    net.cuda()
    net.precision = "bf16"
    X = t(inp["X"]).cuda()
    res = {}
    for wd in ("wide", "narrow"):
        flags.set(bf16_wide=wd == "wide")
        with torch.no_grad():
            res[wd] = net.run(X, keep_all=True, loss_kind=1)
    a, b = res["wide"], res["narrow"]
    for x, y in ((a.Z, b.Z), (a.E, b.E), (a.L, b.L), (a.T, b.T)):
        assert torch.equal(x, y)
    # the per-column partials are summed in a fixed order per slot; the slot layout is the same
    np.testing.assert_allclose(a.loss_sums.cpu().numpy(), b.loss_sums.cpu().numpy(), rtol=1e-6)


@pytest.mark.parametrize("name", sorted(P.BF16_FIXTURES))
def test_bf16_matches_reference_bf16_gemms(name, dl):
    """Against the reference classes themselves run with bf16-operand GEMMs (exact accumulation,
    fp32 state; tests/golden/make_golden_bf16.py) and unmodified in fp32, at bf16_bar with the
    fixture's own yardsticks.  The config-5 fixture (m=1024, n=4096, K=15) runs its full depth."""
    from conftest import load_golden
    import parity
    g, meta = load_golden(name)
    d = meta["defn"]
    inp, sd = P.build_problem(d)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    net = dl.VARIANTS[d["variant"]](m=d["m"], n=0, d=d["n"], batch_size=d["B"], A=t(inp["A"]),
                                    Z0=t(inp["Z0"]), E0=t(inp["E0"]), L0=t(inp["L0"]),
                                    layers=d["K"])
    net.load_state_dict({k: t(v) for k, v in sd.items()})
    net.requires_grad_(False)
    net.precision = "bf16"
    with torch.no_grad():
        out = net(t(inp["X"]).cuda())
    for i, nm in enumerate("ZELT"[:len(out)]):
        for k in range(g[nm].shape[0]):
            got = out[i][k].cpu().numpy()
            s, dk = float(g["s_" + nm][k]), float(g["d_" + nm][k])
            b_bf, b_32 = bf16_bar(s, dk)
            parity.check(name, "bf16", f"{nm}[{k}] vs ref-bf16", nrel(got, g[nm][k]), b_bf, s)
            parity.check(name, "bf16", f"{nm}[{k}] vs ref-f32", nrel(got, g["f32_" + nm][k]),
                         b_32, s)
