"""The fused main_lena.py training objective (net.training_loss(kind="lena"): the fused K-layer
forward + dladmm_lena_f32 + dladmm_bwd_f32 with E / L cotangents) against the same objective built
with torch ops, main_lena.py:221-228 with dual_gap of :145-147:

  * in fp64 on the CPU over the reference-op restatement (oracle/dladmm_torch_cpu.py, pinned to
    the reference classes by tests/test_oracle_torch.py) with torch autograd -- the reference;
  * in fp32 on the GPU over this package's differentiable forward (the reference training loop
    unchanged: torch ops on the returned Z_k, E_k, L_k).

Bar: loss values within 1e-5 (norm-relative, per layer) of fp64; every parameter gradient within
max(GTOL, 3 x the torch-op GPU path's own distance to fp64) -- the GTOL of tests/test_gpu_backward.py
(GEMM summation order and near-threshold shrink masks move fp32 gradients by more than rounding).

The reference's own statements (tests/golden/lena_*.npz: main_lena.py's loss loop and
main_syn_l1l1-dgap_ltheta.py's, executed on the scripts' own classes, make_golden_lena.py) pin
the fused op directly in test_lena_vs_reference_statements.
"""
import os
import sys
from importlib import import_module

import numpy as np
import pytest
import torch

import problems as P

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "oracle"))
import dladmm_torch_cpu as TC  # noqa: E402

GTOL = 1e-4
ALPHA = 0.45  # main_lena.py's alpha


def nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / nb) if nb > 0 else float(np.linalg.norm(a))


from lena_checker import dual_gap, lena_losses  # noqa: E402  (pinned: test_oracle_lena.py)
from conftest import load_golden  # noqa: E402


def build(dl, defn, K):
    d = dict(defn, K=K)
    inp, sd = P.build_problem(d)
    m, n = inp["A"].shape
    B = inp["X"].shape[1]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    net = dl.VARIANTS[d["variant"]](m=m, n=0, d=n, batch_size=B, A=t(inp["A"]),
                                    Z0=t(inp["Z0"]), E0=t(inp["E0"]), L0=t(inp["L0"]), layers=K)
    net.load_state_dict({k: t(v) for k, v in sd.items()}, strict=True)
    return net.cuda(), inp, sd


def fp64_reference(variant, inp, sd, K, coeffs):
    d64 = lambda a: torch.from_numpy(np.asarray(a, np.float64))  # noqa: E731
    params = {k: d64(v).requires_grad_(True) for k, v in sd.items()}
    X, A = d64(inp["X"]), d64(inp["A"])
    fwd = getattr(TC.forward, "__wrapped__", TC.forward)  # the restatement without no_grad
    with torch.enable_grad():
        out = fwd(variant, X, A, d64(inp["Z0"]), d64(inp["E0"]), d64(inp["L0"]), params, K)
        per = lena_losses(out[0], out[1], out[2], X, A, ALPHA, K)
        tot = sum(c * l for c, l in zip(coeffs, per))
        tot.backward()
    return float(tot.detach()), [float(v.detach()) for v in per], \
        {k: p.grad.numpy() for k, p in params.items()}


CASES = [
    ("v1_small_pert", 3),     # shape (32, 32), B = 8
    ("v1_lena_cfg1", 5),      # BASELINE config 1: main_lena.py's shape (64 x 256), B = 20
    ("v1_med_w04", 3),        # config-2 shape (256 x 512), B = 12
    ("v4_med_pert", 3),       # the objective on another variant (any variant takes it)
    ("v2_ragged", 3),         # m = 30, n = 70, B = 5
]


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f32", "f32_split"])
@pytest.mark.parametrize("name,K", CASES, ids=[c[0] for c in CASES])
def test_lena_loss_and_grads_vs_fp64(dl, name, K, precision):
    """At both training precisions: "f32_split" runs V1 (round 6) and V4 on the split-f16 forward
    (V2 falls back to fp32), its saved A Z_k into the reverse sweep and the split-f16 weight
    gradient -- main_lena.py's training step on the f16 matrix cores, at the fp32 bars."""
    defn = P.FIXTURES[name]
    coeffs = [0.6 if k < K - 1 else 1.0 for k in range(K)]
    net, inp, sd = build(dl, defn, K)
    net.requires_grad_(True)
    net.precision = precision
    X = torch.from_numpy(inp["X"]).cuda()
    A = torch.from_numpy(inp["A"]).cuda()
    # fused
    tot_f, per_f = net.training_loss(X, ALPHA, coeffs, kind="lena")
    tot_f.backward()
    g_f = {k: p.grad.detach().cpu().numpy() for k, p in net.named_parameters()}
    # torch ops over the differentiable forward (the reference loop unchanged)
    net.zero_grad(set_to_none=True)
    out = net(X)
    per_t = lena_losses(out[0], out[1], out[2], X, A, ALPHA, K)
    tot_t = sum(c * l for c, l in zip(coeffs, per_t))
    tot_t.backward()
    g_t = {k: p.grad.detach().cpu().numpy() for k, p in net.named_parameters()}
    # fp64 reference
    tot64, per64, g64 = fp64_reference(defn["variant"], inp, sd, K, coeffs)

    assert abs(float(tot_f) - tot64) <= 1e-5 * abs(tot64), (float(tot_f), tot64)
    assert nrel(per_f.detach().cpu().numpy(), per64) <= 1e-5
    worst = []
    for k, g in g64.items():
        if not np.any(g):
            continue
        ef, et = nrel(g_f[k], g), nrel(g_t[k], g)
        bar = max(GTOL, 3 * et)
        worst.append((ef / bar, k, ef, et))
        assert ef <= bar, (k, ef, et)
    worst.sort(reverse=True)
    print(f"{name}: loss {float(tot_f):.8g} vs fp64 {tot64:.8g}; worst grad {worst[0]}")


@pytest.mark.gpu
def test_lena_path_matches_torch_op_path_at_batch(dl):
    """A larger ragged batch at main_lena.py's shape: fused vs torch-op loss on the GPU."""
    defn = dict(P.FIXTURES["v1_lena_cfg1"], B=1000, seed=2201, perturb=0.1, wscale=0.4)
    K = 5
    coeffs = [1.0] * K
    net, inp, _ = build(dl, defn, K)
    net.requires_grad_(True)
    X = torch.from_numpy(inp["X"]).cuda()
    A = torch.from_numpy(inp["A"]).cuda()
    tot_f, per_f = net.training_loss(X, ALPHA, coeffs, kind="lena")
    tot_f.backward()
    g_f = {k: p.grad.detach().double() for k, p in net.named_parameters()}
    net.zero_grad(set_to_none=True)
    out = net(X)
    per_t = lena_losses(out[0], out[1], out[2], X, A, ALPHA, K)
    sum(c * l for c, l in zip(coeffs, per_t)).backward()
    for k, p in net.named_parameters():
        g = p.grad.detach().double()
        e = float((g_f[k] - g).norm() / g.norm().clamp_min(1e-30))
        assert e <= GTOL, (k, e)
    pt = torch.stack([v.detach() for v in per_t]).double()
    assert float((per_f.double() - pt).norm() / pt.norm()) <= 1e-5


def test_lena_descriptor_validation(dl):
    """Host-only: the workspace query rejects what the kernel does not cover (no device work)."""
    import ctypes
    from importlib import import_module
    _lib = import_module("d-ladmm_amd._lib")
    L = _lib.lib()
    d = _lib.LenaDesc()
    d.abi_version = _lib.ABI_VERSION
    d.m, d.n, d.batch, d.layers, d.mode = 64, 256, 100, 3, 0
    d.X = d.A = d.E = d.L = d.sums = 16  # non-null placeholders: never dereferenced here
    d.ld_x = d.ld = 100
    d.ld_a = 256
    d.layer_stride = 64 * 100
    assert L.dladmm_lena_workspace_bytes(ctypes.byref(d)) > 0
    d.n = 600   # past the register-resident shapes
    assert L.dladmm_lena_workspace_bytes(ctypes.byref(d)) == 0
    d.n = 256
    d.mode = 1  # cotangent outputs missing
    assert L.dladmm_lena_workspace_bytes(ctypes.byref(d)) == 0
    d.mode = 0
    d.ld = 50   # row stride below the batch
    assert L.dladmm_lena_workspace_bytes(ctypes.byref(d)) == 0
    # 32-bit offsets over the instantiation's PADDED rows: m = 200 runs on the
    # 256-row instantiation, so ld = 2^21 + 64 passes m*ld*4 < 2^31 but not 256*ld*4
    d.m, d.n = 200, 500
    d.ld_a = 500
    d.batch = d.ld = d.ld_x = (1 << 21) + 64
    d.layer_stride = d.m * d.ld
    assert L.dladmm_lena_workspace_bytes(ctypes.byref(d)) == 0
    d.batch = d.ld = d.ld_x = (1 << 21) - 64 * 40
    d.layer_stride = d.m * d.ld
    assert L.dladmm_lena_workspace_bytes(ctypes.byref(d)) > 0
    # loss-partial rows: 4K rows of the padded batch must stay under 2^31 bytes
    d.layers = 300
    assert L.dladmm_lena_workspace_bytes(ctypes.byref(d)) == 0


def test_lena_host_checks(dl):
    """Host-only: ops.dladmm_lena refuses operands the descriptor cannot describe before any
    launch -- X of another shape than (m, B), A of another row count, host tensors."""
    from importlib import import_module
    ops = import_module("d-ladmm_amd.ops")
    K, m, n, B = 2, 8, 16, 5
    E = torch.zeros(K, m, B)
    L = torch.zeros(K, m, B)
    A = torch.zeros(m, n)
    with pytest.raises(ValueError, match="X must be"):
        ops.dladmm_lena(torch.zeros(m, B + 1), A, E, L, 0.45, B)
    with pytest.raises(ValueError, match="X must be"):
        ops.dladmm_lena(torch.zeros(m, B), torch.zeros(m + 1, n), E, L, 0.45, B)
    with pytest.raises(ValueError, match="one GPU"):
        ops.dladmm_lena(torch.zeros(m, B), A, E, L, 0.45, B)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["v1", "v4"])
def test_lena_column_shards_sum_to_full_batch(variant, dl):
    """Data-parallel shards of the fused main_lena objective (training_loss(kind="lena",
    cols=..., batch=B)): the summed losses and gradients equal the whole batch's."""
    base = "v1_lena_cfg1" if variant == "v1" else "v4_med_pert"
    defn = dict(P.FIXTURES[base], B=96, seed=4411, perturb=0.1, wscale=0.4)
    K, B = 3, 96
    net, inp, sd = build(dl, defn, K)
    net.requires_grad_(True)
    X = torch.from_numpy(inp["X"]).cuda()
    coeffs = [0.6, 0.6, 1.0]
    tf, pf = net.training_loss(X, ALPHA, coeffs, kind="lena")
    tf.backward()
    shard, _, _ = build(dl, defn, K)
    shard.requires_grad_(True)
    tot, per = 0.0, 0.0
    for c0, c1 in (dl.dist.shard_columns(B, 0, 2), dl.dist.shard_columns(B, 1, 2)):
        t, pl = shard.training_loss(X[:, c0:c1], ALPHA, coeffs, kind="lena", batch=B,
                                    cols=(c0, c1))
        t.backward()
        tot, per = tot + float(t), per + pl.double().cpu().numpy()
    np.testing.assert_allclose(tot, float(tf), rtol=1e-5)
    np.testing.assert_allclose(per, pf.double().cpu().numpy(), rtol=1e-5)
    ps = dict(shard.named_parameters())
    for key, p in net.named_parameters():
        e = nrel(ps[key].grad.cpu().numpy(), p.grad.cpu().numpy())
        assert e <= 1e-5, (key, e)


@pytest.mark.gpu
def test_lena_graph_training_step(dl):
    """V1 forward + fused main_lena objective + backward captured as one HIP graph and replayed on
    new data: the objective and every gradient equal an eager step's bit for bit."""
    defn = dict(P.FIXTURES["v1_lena_cfg1"], B=640, seed=4412, perturb=0.1, wscale=0.4)
    K = 4
    net, inp, _ = build(dl, defn, K)
    net.requires_grad_(True)
    X2 = P.make_inputs(defn["m"], defn["n"], defn["B"], 4413)["X"]

    def step(xx):
        total, _ = net.training_loss(xx, ALPHA, [1.0] * K, kind="lena")
        total.backward()
        return total

    def eager(data):
        net.zero_grad(set_to_none=True)
        tot = step(torch.from_numpy(data).cuda()).detach()
        torch.cuda.synchronize()
        return tot, {k: p.grad.clone() for k, p in net.named_parameters()}

    refs = [eager(X2), eager(inp["X"])]
    x = torch.from_numpy(inp["X"]).cuda()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            net.zero_grad(set_to_none=False)
            step(x)
    torch.cuda.current_stream().wait_stream(s)
    net.zero_grad(set_to_none=False)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static_total = step(x)
    for data, (ref_total, ref) in zip((X2, inp["X"]), refs):
        x.copy_(torch.from_numpy(data).cuda())
        for p in net.parameters():
            p.grad.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(static_total.detach(), ref_total)
        for k, p in net.named_parameters():
            assert torch.equal(p.grad, ref[k]), f"grad {k} of the replayed step differs"


@pytest.mark.gpu
def test_lena_upstream_scale_and_eval(dl):
    """The training forward forms the cotangents of sum_k c_k l_k in the same pass as the sums
    (mode 2); the backward multiplies them by the upstream gradient on the device: (2.5 * total)
    .backward() gives 2.5x the gradients, a no-grad evaluation (mode 0) returns the same loss
    values, and a retained graph can be backed through twice."""
    defn = dict(P.FIXTURES["v1_lena_cfg1"], B=200, seed=4421, perturb=0.1, wscale=0.4)
    K = 3
    net, inp, _ = build(dl, defn, K)
    net.requires_grad_(True)
    X = torch.from_numpy(inp["X"]).cuda()
    tot, per = net.training_loss(X, ALPHA, [0.6, 0.6, 1.0], kind="lena")
    tot.backward()
    g1 = {k: p.grad.clone() for k, p in net.named_parameters()}
    for scale in (2.0, 2.5):   # 2: every scaled value exact, so the gradients are exactly 2x
        net.zero_grad(set_to_none=True)
        tot2, _ = net.training_loss(X, ALPHA, [0.6, 0.6, 1.0], kind="lena")
        (scale * tot2).backward()
        for k, p in net.named_parameters():
            if scale == 2.0:
                assert torch.equal(p.grad, 2.0 * g1[k]), k
            else:
                g, r = p.grad.double(), scale * g1[k].double()
                assert float((g - r).norm()) <= 1e-6 * float(r.norm()), k   # some grads are all zero
    with torch.no_grad():
        tot3, per3 = net.training_loss(X, ALPHA, [0.6, 0.6, 1.0], kind="lena")
    assert torch.equal(tot3, tot.detach()) and torch.equal(per3, per.detach())
    # a retained graph backed through twice: the second backward forms the cotangents again
    # (mode 1; the first scaled the forward's in place) -- the gradients accumulate to 2x
    net.zero_grad(set_to_none=True)
    tot4, _ = net.training_loss(X, ALPHA, [0.6, 0.6, 1.0], kind="lena")
    tot4.backward(retain_graph=True)
    tot4.backward()
    for k, p in net.named_parameters():
        g, r = p.grad.double(), 2.0 * g1[k].double()
        assert float((g - r).norm()) <= 1e-6 * float(r.norm()), k


@pytest.mark.gpu
def test_lena_empty_batch(dl):
    """B = 0 (the reference's ops on an empty batch give zero sums): zero sums and empty
    cotangents, no launch."""
    from importlib import import_module
    ops = import_module("d-ladmm_amd.ops")
    K, m, n = 3, 16, 32
    dev = torch.device("cuda", 0)
    E = torch.zeros(K, m, 0, device=dev)
    L = torch.zeros(K, m, 0, device=dev)
    X = torch.zeros(m, 0, device=dev)
    A = torch.randn(m, n, device=dev)
    sm = ops.dladmm_lena(X, A, E, L, 0.45, 1.0)
    assert sm.shape == (K, 4) and not sm.any()
    sm, gE, gL = ops.dladmm_lena(X, A, E, L, 0.45, 1.0, coef=torch.ones(K, device=dev))
    assert not sm.any() and gE.shape == (K, m, 0) and gL.shape == (K, m, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("scale,shape", [(1.0, (64, 256, 37)), (40.0, (64, 256, 37)),
                                         (1.0, (250, 500, 101))],
                         ids=["64x256", "64x256-large", "250x500-ragged"])
def test_lena_op_vs_fp64_incl_large_arguments(dl, scale, shape):
    """dladmm_lena (mode 2) against fp64 torch: the four sums and the E / L cotangents, with L
    scaled so that many |A^T L| and |L| pass 30 (the linear branch; e^|y| squared overflows there
    and must be discarded by the select, not leak as inf / NaN); and a ragged shape (m, n not
    multiples of 16, B not of 64) whose padded rows and columns must contribute nothing."""
    from importlib import import_module
    ops = import_module("d-ladmm_amd.ops")
    dev = torch.device("cuda", 0)
    K = 2
    m, n, B = shape
    g = torch.Generator().manual_seed(4431)
    X = torch.randn(m, B, generator=g, dtype=torch.float64)
    A = torch.randn(m, n, generator=g, dtype=torch.float64) / 8
    E = torch.randn(K, m, B, generator=g, dtype=torch.float64) * 0.1
    E[:, :3] = 0.0   # sgn(0) = 0
    L = torch.randn(K, m, B, generator=g, dtype=torch.float64) * scale
    X, A, E, L = (t.float().double() for t in (X, A, E, L))  # the fp32 operands, exactly
    c = torch.tensor([0.6, 1.0], dtype=torch.float64)
    f = lambda t: t.float().to(dev)  # noqa: E731
    sm, gE, gL = ops.dladmm_lena(f(X), f(A), f(E), f(L), ALPHA, B, coef=f(c))
    Xd, Ad = X, A
    Ed, Ld = E.clone().requires_grad_(True), L.clone().requires_grad_(True)
    Y = torch.einsum("mn,kmb->knb", Ad, Ld)
    ref = torch.stack([Ed.abs().sum((1, 2)), dual_gap(Y, ALPHA).sum((1, 2)),
                       dual_gap(Ld, 1).sum((1, 2)), (Ld * Xd).sum((1, 2))], 1)
    assert torch.isfinite(sm).all() and torch.isfinite(gE).all() and torch.isfinite(gL).all()
    sc = ref.detach().abs().sum(0)  # per-term scale
    assert float(((sm.cpu() - ref.detach()).abs().max(0).values / sc).max()) <= 1e-5
    loss = (c * (ref[:, 0] / (m * B) + ref[:, 1] / (n * B) + (ref[:, 2] + ref[:, 3]) / (m * B))).sum()
    loss.backward()
    assert nrel(gE.cpu(), Ed.grad) <= 1e-5
    assert nrel(gL.cpu(), Ld.grad) <= 1e-5


LENA_NAMES = sorted(P.LENA_FIXTURES)


@pytest.mark.gpu
@pytest.mark.parametrize("name", LENA_NAMES)
def test_lena_vs_reference_statements(dl, name):
    """training_loss(kind="lena") against the reference scripts' own loss loop + backward
    (fixtures): main_lena.py (+ mean(L X), every layer, alpha 0.45) and
    main_syn_l1l1-dgap_ltheta.py (- mean(L X), only the last layer, alpha 0.01, V2 at 250 x 500).
    Total and per-layer values within max(1e-5, 2 x the reference's fp32-vs-fp64 gap) of the
    reference's fp64 run; every gradient within max(GTOL, 3 x its fp32-vs-fp64 gap) of the
    reference's fp32 gradient (the bar of tests/test_gpu_backward.py)."""
    g, meta = load_golden(name)
    d = meta["defn"]
    K = d["K"]
    start = meta["loss_start_layer"]
    coeffs = [0.0 if k < start else 1.0 for k in range(K)]
    net, inp, sd = build(dl, d, K)
    net.requires_grad_(True)
    X = torch.from_numpy(inp["X"]).cuda()
    tot, per = net.training_loss(X, meta["alpha"], coeffs, kind="lena", lx_sign=meta["lx_sign"])
    tot.backward()
    t32, t64 = (float(v) for v in g["total"])
    assert abs(float(tot) - t64) <= max(1e-5 * abs(t64), 2 * abs(t32 - t64)), (float(tot), t64)
    p32, p64 = g["per_layer"]
    mine = per.detach().double().cpu().numpy()[start:]
    e = nrel(mine, p64[start:])
    assert e <= max(1e-5, 2 * nrel(p32[start:], p64[start:])), e
    worst = []
    for key, p in net.named_parameters():
        ref = g["g:" + key]
        gm = np.zeros_like(ref) if p.grad is None else p.grad.detach().cpu().numpy()
        if not np.any(ref):
            assert not np.any(gm), key
            continue
        err = nrel(gm, ref)
        bar = max(GTOL, 3 * float(g["gap:" + key]))
        worst.append((err / bar, key, err))
        assert err <= bar, (key, err, bar)
    worst.sort(reverse=True)
    print(f"{name}: total {float(tot):.8g} vs ref fp64 {t64:.8g}; worst grad {worst[0]}")


@pytest.mark.gpu
@pytest.mark.parametrize("lx_sign", [1.0, -1.0])
def test_lena_cotangents_in_backward_bit_equal(dl, lx_sign):
    """save_cotangents=False (mode 0 forward, mode 1 backward: no 2 K m B cotangent buffers held
    between forward and backward) gives the same loss and gradients bit for bit as the default
    mode-2 forward, for either sign of the L X term."""
    defn = dict(P.FIXTURES["v1_lena_cfg1"], B=200, seed=4441, perturb=0.1, wscale=0.4)
    K = 3
    net, inp, _ = build(dl, defn, K)
    net.requires_grad_(True)
    X = torch.from_numpy(inp["X"]).cuda()
    res = []
    for save in (True, False):
        net.zero_grad(set_to_none=True)
        tot, per = net.training_loss(X, ALPHA, [0.6, 0.6, 1.0], kind="lena", lx_sign=lx_sign,
                                     save_cotangents=save)
        tot.backward()
        res.append((tot.detach(), per.detach(),
                    {k: p.grad.clone() for k, p in net.named_parameters()}))
    (t0, p0, g0), (t1, p1, g1) = res
    assert torch.equal(t0, t1) and torch.equal(p0, p1)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k


@pytest.mark.gpu
def test_lena_evaluation_any_precision(dl):
    """No parameter needs a gradient: training_loss(kind="lena") evaluates at the module's
    precision (bf16 included, which training refuses) and equals the training forward's values
    at f32."""
    defn = dict(P.FIXTURES["v1_lena_cfg1"], B=300, seed=4451, perturb=0.1, wscale=0.4)
    K = 3
    net, inp, _ = build(dl, defn, K)
    X = torch.from_numpy(inp["X"]).cuda()
    net.requires_grad_(True)
    tot_t, per_t = net.training_loss(X, ALPHA, [0.6, 0.6, 1.0], kind="lena", lx_sign=-1.0)
    net.requires_grad_(False)
    tot_e, per_e = net.training_loss(X, ALPHA, [0.6, 0.6, 1.0], kind="lena", lx_sign=-1.0)
    assert torch.equal(tot_e, tot_t.detach()) and torch.equal(per_e, per_t.detach())
    net.precision = "bf16"
    tot_b, per_b = net.training_loss(X, ALPHA, [0.6, 0.6, 1.0], kind="lena", lx_sign=-1.0)
    assert torch.isfinite(per_b).all()
    assert float((per_b.double() - per_e.double()).norm() / per_e.double().norm()) <= 2e-2
    net.requires_grad_(True)
    with pytest.raises(RuntimeError, match="inference-only"):
        net.training_loss(X, ALPHA, [0.6, 0.6, 1.0], kind="lena")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sums", "grads", "both"])
def test_lena_rowsplit_kernel_matches_64_column_kernel(dl, mode):
    """dladmm_lena_f32 at a small batch runs the row-split kernel (16 columns per workgroup,
    rows over the 4 waves); at a batch past one workgroup per CU the 64-column one.  Columns are
    independent, so the first 20 columns of a 4,200-column call are the 20-column call: gE, gL
    bit for bit; the sums (the same terms added in another order) within 1e-6."""
    ops = import_module("d-ladmm_amd.ops")
    g = torch.Generator(device="cuda").manual_seed(77)
    m, n, K, Bs, Bb = 256, 512, 3, 20, 4200
    A = torch.randn(m, n, generator=g, device="cuda") / 16
    X = torch.randn(m, Bb, generator=g, device="cuda")
    E = torch.randn(K, m, Bb, generator=g, device="cuda") * 0.3
    L = torch.randn(K, m, Bb, generator=g, device="cuda") * 0.5
    coef = torch.rand(K, generator=g, device="cuda") if mode != "sums" else None
    kw = dict(coef=coef, sums=mode != "grads")
    small = ops.dladmm_lena(X[:, :Bs].contiguous(), A, E[:, :, :Bs].contiguous(),
                            L[:, :, :Bs].contiguous(), 0.45, Bs, **kw)
    big = ops.dladmm_lena(X, A, E, L, 0.45, Bs, **kw)
    if mode == "sums":
        small, big = (small,), (big,)
    if mode != "sums":
        gE_s, gL_s = small[-2], small[-1]
        gE_b, gL_b = big[-2], big[-1]
        assert torch.equal(gE_s, gE_b[:, :, :Bs]) and torch.equal(gL_s, gL_b[:, :, :Bs])
    if mode != "grads":
        # the big call's sums cover 4,200 columns: compare the small one with an fp64 restatement
        # of its own 20 columns instead (dual_gap in closed form, main_lena.py:145-147)
        import torch.nn.functional as F
        Xd, Ad = X[:, :Bs].double(), A.double()
        ref = []
        for k in range(K):
            Ek, Lk = E[k, :, :Bs].double(), L[k, :, :Bs].double()
            dg = lambda x, c: F.softplus(x - c) + F.softplus(-x - c)  # noqa: E731
            ref.append([Ek.abs().sum(), dg(Ad.t() @ Lk, 0.45).sum(), dg(Lk, 1.0).sum(),
                        (Lk * Xd).sum(), (Lk * Xd).abs().sum()])
        got = small[0].cpu().numpy()
        ref = np.array([[float(v) for v in r] for r in ref])
        np.testing.assert_allclose(got[:, :3], ref[:, :3], rtol=1e-5)
        # sum L X cancels: its bar is relative to the sum of the terms' magnitudes
        assert np.all(np.abs(got[:, 3] - ref[:, 3]) <= 1e-5 * ref[:, 4])
