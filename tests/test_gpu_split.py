"""Parity of the split-f16 fused forward (precision "f32_split", DLADMM_PREC_F32_SPLIT,
csrc/dladmm_fused_x3.hip) with the reference -- the SAME bars as the fp32 path
(tests/test_gpu_parity.py, tests/parity.py): per layer, norm-relative <= max(1e-5, 2 x the
reference's own
fp32-vs-fp64 gap), against the reference's golden outputs and the oracle.

The mode forms every fp32 GEMM as hi*hi + hi*lo + lo*hi of exactly split, power-of-two-scaled f16
halves with fp32 accumulation; these tests are what pins that its error is an fp32 GEMM's:
every variant it runs (V1 with its per-sample betas since round 6, V4, V5, V6 and the newS
schedules on them), padded shapes, ragged batches,
the 65,536-column BASELINE shape, columns of very different magnitude (per-column scaling, the
provisional-scale re-split), lean mode and determinism.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
import problems as P
import parity
from test_gpu_parity import REL, _compare, _oracle_case, check_golden, make_net, nrel

pytestmark = pytest.mark.gpu

SPLIT_VARIANTS = ("v1", "v4", "v5", "v6", "v7", "v7t", "v7p")


def split_net(dl, variant, inp, sd, K, **extra):
    net = make_net(dl, variant, inp, sd, K, **extra)
    net.precision = "f32_split"
    return net


def _path(dl, net, X):
    """The C ABI's plan for this call (4 = split-f16 fused kernel)."""
    import ctypes
    from importlib import import_module
    ops = import_module("d-ladmm_amd.ops")
    d = dl._lib.FwdDesc()
    m, B = X.shape
    K = net.layers
    out = ops.ForwardResult(torch.empty(K, net.d, B, device="cuda"),
                            torch.empty(K, m, B, device="cuda"),
                            torch.empty(K, m, B, device="cuda"),
                            torch.empty(K + 1, m, B, device="cuda"), None)
    tabs = dict(scalar_params=None, row_params=None, beta1_elem=(), beta2_elem=())
    tabs.update(net._tables(net.A.device))
    keep = ops._fill_fwd_desc(d, net.VARIANT, X, net.A, [w.detach() for w in net._weights()],
                              net.Z0, net.E0, net.L0, keep_all=True, loss_kind=0, out=out,
                              **tabs)
    d.precision = dl._lib.PREC_F32_SPLIT
    del keep
    return dl._lib.lib().dladmm_fwd_path(ctypes.byref(d))


@pytest.mark.parametrize("name", sorted(n for n in P.FIXTURES
                                        if P.FIXTURES[n]["variant"] in SPLIT_VARIANTS))
def test_split_matches_reference_golden(name, dl):
    g, meta = load_golden(name)
    d = meta["defn"]
    inp, sd = P.build_problem(d)
    net = split_net(dl, d["variant"], inp, sd, d["K"], **P.ctor_extra(d))
    X = torch.from_numpy(inp["X"]).cuda()
    if d["m"] <= 256 and d["n"] <= 512 and d["B"] % 4 == 0:
        assert _path(dl, net, X) == 4
    with torch.no_grad():
        out = net(X)
    check_golden(name, g, meta, net, X, out, path="split")


@pytest.mark.parametrize("variant", ["v1", "v4", "v5", "v6"])
@pytest.mark.parametrize("B", [1, 64, 300])
def test_split_vs_oracle_baseline_shape(variant, B, dl, oracle):
    m, n, K = 256, 512, 15
    inp, sd, ref = _oracle_case(oracle, variant, m, n, B, K, seed=2000 + B,
                                wscale=0.4 if variant == "v1" else None)
    net = split_net(dl, variant, inp, sd, K)
    with torch.no_grad():
        out = net(torch.from_numpy(inp["X"]).cuda())
    _compare(out, ref, tag=f"split {variant} B={B}", path="split")


@pytest.mark.parametrize("shape", [(16, 32), (30, 70), (64, 256), (250, 500), (200, 512)])
def test_split_padded_shapes(shape, dl, oracle):
    m, n = shape
    for variant in ("v4", "v6", "v1"):   # V1: per-sample betas read past the last row as 0
        inp, sd, ref = _oracle_case(oracle, variant, m, n, 76, 5, seed=3000 + m,
                                    wscale=0.4 if variant == "v1" else None)
        net = split_net(dl, variant, inp, sd, 5)
        assert _path(dl, net, torch.from_numpy(inp["X"]).cuda()) == 4
        with torch.no_grad():
            out = net(torch.from_numpy(inp["X"]).cuda())
        _compare(out, ref, tag=f"split {variant} {shape}", path="split")


def test_split_column_magnitudes(dl, oracle):
    """Columns scaled by 1e-6 .. 1e6 (and an all-zero column): the per-column power-of-two
    scales keep every column at the top of the f16 range; Z growing by far more than the
    provisional scale's headroom between layers takes the exact re-split."""
    m, n, B, K = 256, 512, 64, 6
    inp = P.make_inputs(m, n, B, 4100)
    scales = (10.0 ** np.linspace(-6, 6, B)).astype(np.float32)
    scales[7] = 0.0
    inp = dict(inp, X=inp["X"] * scales, Z0=inp["Z0"] * scales)
    sd = P.make_state_dict("v6", m, n, B, K, inp["A"], 4100, perturb=0.1)
    for k in range(K):   # thresholds scaled like the data would need: keep them tiny
        sd[f"active_para.{k}"][:] = 1e-7
    args = ("v6", inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, K)
    r64 = oracle.forward(*args, dtype=np.float64)
    net = split_net(dl, "v6", inp, sd, K)
    with torch.no_grad():
        Z, E, L, T = net(torch.from_numpy(inp["X"]).cuda())
    for nm, seq in (("Z", Z), ("E", E), ("L", L)):
        for k in range(K):
            got = seq[k].cpu().numpy().astype(np.float64)
            ref = np.asarray(r64[nm][k], np.float64)
            # per column: every column matches at its own scale
            for c in range(B):
                nr = np.linalg.norm(ref[:, c])
                if nr == 0:
                    assert np.all(got[:, c] == 0), (nm, k, c)
                    continue
                e = np.linalg.norm(got[:, c] - ref[:, c]) / nr
                assert e <= 1e-5, (nm, k, c, e)


def test_split_lean_mode_and_determinism(dl):
    """Lean mode (Z_k through the ping-pong workspace) == the full run's last layer, bitwise;
    two runs bitwise identical."""
    m, n, B, K = 256, 512, 1000, 15
    inp = P.make_inputs(m, n, B, 5001)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 5001, perturb=0.1)
    net = split_net(dl, "v4", inp, sd, K)
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


def test_split_baseline_size(dl, oracle):
    """B = 65,536: a random column subset against the oracle, the fused objective against a
    separate fp64 reduction of the returned outputs, and against the fp32 path."""
    m, n, K, B = 256, 512, 15, 65536
    inp = P.make_inputs(m, n, 64, 8001)
    A = inp["A"]
    rng = np.random.default_rng(8002)
    zs = (rng.random((n, B)) < 0.1) * rng.standard_normal((n, B))
    es = (rng.random((m, B)) < 0.1) * rng.standard_normal((m, B))
    X = (A.astype(np.float64) @ zs + es).astype(np.float32)
    Z0 = (rng.random((n, B)) / n).astype(np.float32)
    E0 = np.zeros((m, B), np.float32)
    L0 = np.zeros((m, B), np.float32)
    sd = P.make_state_dict("v4", m, n, B, K, A, 8001, perturb=0.1)
    net = split_net(dl, "v4", dict(A=A, X=X, Z0=Z0, E0=E0, L0=L0), sd, K)
    Xd = torch.from_numpy(X).cuda()
    with torch.no_grad():
        r, obj = net.layer_objectives(Xd, 0.001, "l1l1")
        net.precision = "f32"
        r32, obj32 = net.layer_objectives(Xd, 0.001, "l1l1")
    cols = np.sort(np.random.default_rng(8003).permutation(B)[:96])
    ref = oracle.forward("v4", X[:, cols], A, Z0[:, cols], E0[:, cols], L0[:, cols], sd, K)
    for nm, got, g32 in (("Z", r.Z, r32.Z), ("E", r.E, r32.E), ("L", r.L, r32.L)):
        for k in range(K):
            parity.check("v4 B=65536 columns", "split", f"{nm}[{k}] vs oracle32",
                         nrel(got[k][:, cols].cpu().numpy(), ref[nm][k]), REL)
            parity.check("v4 B=65536", "split", f"{nm}[{k}] vs f32 path",
                         nrel(got[k].cpu().numpy(), g32[k].cpu().numpy()), REL)
    Ad = torch.from_numpy(A).cuda().double()
    sep = []
    for k in range(K):
        Zk = r.Z[k].double()
        sep.append(float((0.001 * Zk.abs().sum() + (Xd.double() - Ad @ Zk).abs().sum()) / B))
    np.testing.assert_allclose(obj.cpu().numpy(), np.array(sep), rtol=1e-5)
    np.testing.assert_allclose(obj.cpu().numpy(), obj32.cpu().numpy(), rtol=1e-5)


def test_split_falls_back_where_unsupported(dl, oracle):
    """V2-V3, shapes beyond the register budget and batches that are not a multiple of 4 run the
    fp32 kernels under f32_split."""
    for variant, (m, n), B in (("v1", (64, 256), 50), ("v3", (64, 256), 52),
                               ("v4", (300, 600), 52), ("v4", (256, 512), 50)):
        inp, sd, ref = _oracle_case(oracle, variant, m, n, B, 3, seed=3100,
                                    wscale=0.4 if variant == "v1" else None)
        net = split_net(dl, variant, inp, sd, 3)
        X = torch.from_numpy(inp["X"]).cuda()
        assert _path(dl, net, X) in (1, 2)
        with torch.no_grad():
            out = net(X)
        _compare(out, ref, tag=f"split fallback {variant}")
    net.requires_grad_(True)
    out = net(X)          # f32_split trains (here on the fp32 fallback kernels)
    assert out[0][0].requires_grad
    net.precision = "bf16"
    with pytest.raises(RuntimeError, match="inference-only"):
        net(X)


@pytest.mark.parametrize("variant", ["v1", "v4", "v5", "v6"])
def test_split_training_saves_product_and_matches_fp32(variant, dl):
    """Training on the split-f16 forward: it stores P_k = A Z_k (the product its E / L / T updates
    consumed), so the backward runs the reverse sweep on it; the gradients of the fused objective
    equal the fp32 path's within the backward tests' GTOL (tests/test_gpu_backward.py), both runs
    on the same parameters and data, and the saved P equals A Z_k to fp32 GEMM accuracy."""
    from importlib import import_module
    ops = import_module("d-ladmm_amd.ops")
    from test_gpu_backward import make_train_net
    m, n, B, K = 256, 512, 200, 4
    inp = P.make_inputs(m, n, B, 7711)
    # V1 at W = 0.4 (A^T + 1e-3 N): its default init is the ill-conditioned case
    sd = P.make_state_dict(variant, m, n, B, K, inp["A"], 7711, perturb=0.1,
                           wscale=0.4 if variant == "v1" else None)
    X = torch.from_numpy(inp["X"]).cuda()
    kind = "lasso" if variant == "v6" else "l1l1"
    coeffs = [0.6] * (K - 1) + [1.0]
    grads, tots = {}, {}
    for prec in ("f32", "f32_split"):
        net = make_train_net(dl, variant, inp, sd, K)
        net.precision = prec
        tot, _ = net.training_loss(X, 1e-3, coeffs, kind)
        tot.backward()
        tots[prec] = float(tot.detach())
        grads[prec] = {k: p.grad.detach().double().cpu().numpy() for k, p in net.named_parameters()
                       if p.grad is not None}
    assert abs(tots["f32_split"] - tots["f32"]) <= 1e-5 * abs(tots["f32"])
    assert grads["f32"].keys() == grads["f32_split"].keys()
    for k, g in grads["f32"].items():
        assert nrel(grads["f32_split"][k], g) <= 1e-4, k
    # the saved product and the plan
    net = make_train_net(dl, variant, inp, sd, K)
    net.precision = "f32_split"
    W = [w.detach() for w in net._weights()]
    r = ops.dladmm_forward(net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0, keep_all=True,
                           want_T=True, want_P=True, precision="f32_split",
                           **net._tables(net.A.device))
    assert r.path == 4 and r.P is not None
    Pref = torch.stack([net.A.double() @ r.Z[k].double() for k in range(K)])
    assert float((r.P.double() - Pref).norm() / Pref.norm()) < 1e-6
    res = ops.dladmm_backward(net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0, r,
                              gZ=[torch.ones_like(r.Z[k]) for k in range(K)],
                              tied=net._shared_weight(), **net._tables(net.A.device))
    assert res.path == 1


@pytest.mark.parametrize("variant", ["v4", "v5", "v6"])
def test_split_weight_gradient_on_f16_cores(variant, dl, flags):
    """Under precision "f32_split" the backward's weight-gradient GEMM (gU_k Var_k^T over the
    batch) also runs on the f16 matrix cores with exactly split operands
    (csrc/dladmm_wgrad_x3.hip): its gradients equal the fp32-MFMA kernel's (plan flag
    wgrad_f32) within fp32 GEMM accuracy, every other gradient is unchanged bitwise, and it is
    deterministic.  B = 4,096: whole 32-column sub-chunks of the split-K chunks."""
    from test_gpu_backward import make_train_net
    m, n, B, K = 256, 512, 4096, 3
    inp = P.make_inputs(m, n, B, 7713)
    sd = P.make_state_dict(variant, m, n, B, K, inp["A"], 7713, perturb=0.1)
    X = torch.from_numpy(inp["X"]).cuda()
    kind = "lasso" if variant == "v6" else "l1l1"
    coeffs = [0.6] * (K - 1) + [1.0]
    grads = {}
    for mode in ("0", "1", "1b"):
        flags.set(wgrad_f32=mode == "0")
        net = make_train_net(dl, variant, inp, sd, K)
        net.precision = "f32_split"
        tot, _ = net.training_loss(X, 1e-3, coeffs, kind)
        tot.backward()
        torch.cuda.synchronize()
        grads[mode] = {k: p.grad.detach().clone() for k, p in net.named_parameters()
                       if p.grad is not None}
    assert grads["0"].keys() == grads["1"].keys()
    # the weights' gradients and V5's ss1 (its gradient is <W, gU Var^T> of the same sums)
    wkeys = [k for k in grads["0"] if k.startswith(("fc", "ss1"))]
    assert wkeys
    # the split-f16 GEMM ran: a different rounding sequence of the same sums
    assert any(not torch.equal(grads["1"][k], grads["0"][k]) for k in wkeys)
    for k in grads["0"]:
        assert torch.equal(grads["1"][k], grads["1b"][k]), k  # deterministic
        a, b = grads["1"][k].double(), grads["0"][k].double()
        if k in wkeys:
            assert float((a - b).norm() / b.norm()) <= 1e-5, k
        else:
            assert torch.equal(grads["1"][k], grads["0"][k]), k


@pytest.mark.parametrize("B", [20, 100, 300])
def test_split_weight_gradient_any_batch(B, dl, flags):
    """Every batch takes the split-f16 weight gradient on the reverse sweep (its operand columns
    are padded to 32 and its chunks rounded to whole 32-column sub-chunks), including the
    reference's batch_size = 20 (main_lena.py:155): fc* gradients within 1e-5 of the fp32-MFMA
    kernel's and not bitwise equal to them (the f16 kernel ran)."""
    from test_gpu_backward import make_train_net
    m, n, K = 256, 512, 3
    inp = P.make_inputs(m, n, B, 7715)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 7715, perturb=0.1)
    X = torch.from_numpy(inp["X"]).cuda()
    grads = {}
    for mode in ("0", "1"):
        flags.set(wgrad_f32=mode == "0")
        net = make_train_net(dl, "v4", inp, sd, K)
        net.precision = "f32_split"
        tot, _ = net.training_loss(X, 1e-3, [0.6, 0.6, 1.0], "l1l1")
        tot.backward()
        grads[mode] = {k: p.grad.detach().clone() for k, p in net.named_parameters()
                       if p.grad is not None and k.startswith("fc")}
    for k, b in grads["0"].items():
        a = grads["1"][k]
        assert not torch.equal(a, b), k
        assert float((a.double() - b.double()).norm() / b.double().norm()) <= 1e-5, k


@pytest.mark.parametrize("m,n,ramp", [(256, 512, False), (64, 256, False), (256, 512, True),
                                      (64, 256, True)])
def test_split_weight_gradient_full_batch(m, n, ramp, dl, flags):
    """The split-f16 weight gradient at the bench's batch (B = 65,536: 32 sub-chunks per split-K
    chunk, multi-GiB operand buffers whose addresses cross bit 31) in both V-tile widths (m = 256:
    256-row tiles, three buffers; m = 64 (rows padded to 128): 128-row tiles, two workgroups per
    CU): the fc*
    gradients stay within 1e-5 of the fp32-MFMA kernel's.  ramp: X's columns grow by 2^12 across
    every 1,024-column chunk, so the running scales drop many times inside a chunk (each an exact
    power-of-two rescale of the accumulators)."""
    from test_gpu_backward import make_train_net
    B, K = 65536, 2
    inp = P.make_inputs(m, n, B, 7717)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 7717, perturb=0.1)
    X = torch.from_numpy(inp["X"]).cuda()
    if ramp:
        X = X * torch.exp2(12.0 * (torch.arange(B, device=X.device) % 1024) / 1024 - 6.0)
    grads = {}
    for mode in ("0", "1"):
        flags.set(wgrad_f32=mode == "0")
        net = make_train_net(dl, "v4", inp, sd, K)
        net.precision = "f32_split"
        tot, _ = net.training_loss(X, 1e-3, [0.6, 1.0], "l1l1")
        tot.backward()
        torch.cuda.synchronize()
        grads[mode] = {k: p.grad.detach().clone() for k, p in net.named_parameters()
                       if p.grad is not None and k.startswith("fc")}
        del net, tot
    assert grads["0"]
    for k, b in grads["0"].items():
        a = grads["1"][k].double()
        assert torch.isfinite(a).all(), k
        assert float((a - b.double()).norm() / b.double().norm()) <= 1e-5, k


def test_split_weight_gradient_per_layer_backward(dl, flags):
    """The per-layer backward (plan flag bwd_per_layer: the fallback when the reverse sweep's
    workspace does not fit) also runs the weight-gradient GEMM split-f16 after a split-f16
    forward: fc* gradients within 1e-5 of the fp32-MFMA kernel's and not bitwise equal to them;
    every other gradient bitwise equal."""
    from test_gpu_backward import make_train_net
    m, n, B, K = 256, 512, 4096, 3
    inp = P.make_inputs(m, n, B, 7719)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 7719, perturb=0.1)
    X = torch.from_numpy(inp["X"]).cuda()
    flags.set(bwd_per_layer=True)
    grads = {}
    for mode in ("0", "1"):
        flags.set(wgrad_f32=mode == "0")
        net = make_train_net(dl, "v4", inp, sd, K)
        net.precision = "f32_split"
        tot, _ = net.training_loss(X, 1e-3, [0.6, 0.6, 1.0], "l1l1")
        tot.backward()
        torch.cuda.synchronize()
        grads[mode] = {k: p.grad.detach().clone() for k, p in net.named_parameters()
                       if p.grad is not None}
    wkeys = [k for k in grads["0"] if k.startswith("fc")]
    assert wkeys
    assert any(not torch.equal(grads["1"][k], grads["0"][k]) for k in wkeys)
    for k in grads["0"]:
        a, b = grads["1"][k].double(), grads["0"][k].double()
        if k in wkeys:
            assert float((a - b).norm() / b.norm()) <= 1e-5, k
        else:
            assert torch.equal(grads["1"][k], grads["0"][k]), k


@pytest.mark.parametrize("side", ["G", "V"])
def test_split_weight_gradient_row_range(side, dl, flags):
    """Per-row accuracy of the split-f16 weight gradient (csrc/dladmm_wgrad_x3.hip "Dynamic
    range"): its power-of-two scales are per wave (64 G rows x 64 V rows), so rows far below the
    wave's largest lose low-order bits.  Here every other row of one operand is 2^20 below its
    neighbours (G = gU_0: rows of the cotangent of Z_0; V = Var_0: rows of E0, with X = Z0 = L0
    = 0 so Var_0 = beta1 E0), and EVERY row of gW (G side) / column (V side) must match the
    fp32-MFMA kernel within 1e-5 of that row's own norm -- the documented per-wave range."""
    from importlib import import_module
    ops = import_module("d-ladmm_amd.ops")
    from test_gpu_backward import make_train_net
    m, n, B, K = 256, 512, 4096, 1
    rng = np.random.default_rng(7731)
    A = P.make_inputs(m, n, 4, 7731)["A"]
    E0 = rng.standard_normal((m, B)).astype(np.float32)
    gz = rng.standard_normal((n, B)).astype(np.float32)
    if side == "G":
        gz[1::2] *= 2.0 ** -20
    else:
        E0[1::2] *= 2.0 ** -20
    z = np.zeros
    inp = dict(A=A, X=z((m, B), np.float32), Z0=z((n, B), np.float32), E0=E0,
               L0=z((m, B), np.float32))
    sd = P.make_state_dict("v4", m, n, B, K, A, 7731, perturb=0.1)
    sd["active_para.0"][:] = 0.0   # every element of Z_0 passes the shrink: gU_0 = gZ_0
    net = make_train_net(dl, "v4", inp, sd, K)
    X = torch.from_numpy(inp["X"]).cuda()
    W = [w.detach() for w in net._weights()]
    tabs = net._tables(net.A.device)
    with torch.no_grad():
        r = ops.dladmm_forward(net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0, keep_all=True,
                               want_T=True, want_P=True, precision="f32_split", **tabs)
    assert r.path == 4
    gZ = [torch.from_numpy(gz).cuda()]
    res = {}
    for f32 in (True, False):
        flags.set(wgrad_f32=f32)
        res[f32] = ops.dladmm_backward(net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0, r,
                                       gZ=gZ, **tabs).gW[0].double()
    a, b = res[False], res[True]
    assert not torch.equal(a, b)
    dim = 1 if side == "G" else 0          # gW is (n, m): G rows are its rows, V rows its columns
    err = ((a - b).norm(dim=dim) / b.norm(dim=dim)).cpu().numpy()
    assert np.all(err <= 1e-5), (side, float(err.max()), int(err.argmax()))
