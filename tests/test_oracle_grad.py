"""The backward oracle (oracle/dladmm_oracle_grad.py, a hand-written reverse sweep) is pinned
against gradients the reference classes produce under torch autograd
(tests/golden/make_golden_grad.py).  CPU only."""
import numpy as np
import pytest

from conftest import load_golden
import problems as P


def grad_case(name, oracle_grad, dtype=np.float32):
    g, meta = load_golden(name)
    d = meta["defn"]
    inp, sd = P.build_problem(d)
    ret_t = P.VARIANT_SPECS[d["variant"]]["ret_t"]
    up = P.make_upstream(d, ret_t)
    return g, meta, d, inp, sd, up


def oracle_grads(og, d, inp, sd, up, kind, dtype=np.float32):
    from oracle import dladmm_oracle as fwd
    out = fwd.forward(d["variant"], inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, d["K"],
                      dtype=dtype)
    gz = og.train_loss_grads(out["Z"], inp["X"], inp["A"], P.GRAD_ALPHA, P.loss_coeffs(d["K"]),
                             kind, dtype=dtype)
    gz = [a + b for a, b in zip(gz, up["Gz"])]
    return og.vjp(d["variant"], inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, d["K"],
                  gZ=gz, gE=list(up["Ge"]), gL=list(up["Gl"]),
                  gT=list(up["Gt"]) if "Gt" in up else None, dtype=dtype)


@pytest.fixture(scope="module")
def og():
    from oracle import dladmm_oracle_grad
    return dladmm_oracle_grad


@pytest.mark.parametrize("name", sorted(P.GRAD_FIXTURES))
def test_upstream_regenerates(name):
    g, meta = load_golden(name)
    d = meta["defn"]
    up = P.make_upstream(d, P.VARIANT_SPECS[d["variant"]]["ret_t"])
    assert {k: P.sha256(v) for k, v in up.items()} == meta["sha256"]
    _, sd = P.build_problem(d)
    assert list(sd.keys()) == meta["keys"]


@pytest.mark.parametrize("name", sorted(P.GRAD_FIXTURES))
def test_grad_oracle_matches_reference_autograd(name, og):
    g, meta, d, inp, sd, up = grad_case(name, og)
    got = oracle_grads(og, d, inp, sd, up, meta["gdef"]["loss"])
    for k in meta["keys"]:
        ref = g["g:" + k]
        assert got[k].shape == ref.shape, k
        # same fp32 op sequence; only BLAS summation order differs from torch's
        tol = max(2e-5, 3.0 * float(g["gap:" + k]))
        e = P_nrel(got[k], ref)
        assert e <= tol, (k, e, tol)


def test_grad_oracle_fp64_matches_finite_differences(og):
    """Independent of the reference: the fp64 reverse sweep agrees with central differences of
    the fp64 forward on a tiny V4 problem (checks the derivation itself)."""
    from oracle import dladmm_oracle as fwd
    d = dict(variant="v4", m=6, n=10, B=3, K=2, seed=77, perturb=0.2)
    inp, sd = P.build_problem(d)
    rng = np.random.default_rng(5)
    G = {nm: [rng.standard_normal(s) for _ in range(d["K"] + (nm == "T"))]
         for nm, s in (("Z", (10, 3)), ("E", (6, 3)), ("L", (6, 3)), ("T", (6, 3)))}

    def f(sdx):
        o = fwd.forward("v4", inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sdx, d["K"],
                        dtype=np.float64)
        return sum(float((G[nm][k] * o[nm][k]).sum()) for nm in G for k in range(len(G[nm])))

    gr = og.vjp("v4", inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, d["K"],
                gZ=G["Z"], gE=G["E"], gL=G["L"], gT=G["T"], dtype=np.float64)
    h = 1e-6
    for key in ("beta1.0", "beta2.1", "beta3.0", "ss2.1", "active_para.0", "active_para1.1"):
        sp = {k: v.astype(np.float64) for k, v in sd.items()}
        sm = {k: v.astype(np.float64) for k, v in sd.items()}
        sp[key] = sp[key] + h
        sm[key] = sm[key] - h
        fd = (f(sp) - f(sm)) / (2 * h)
        assert abs(fd - float(gr[key].sum())) <= 1e-5 * max(1.0, abs(fd)), key
    sp = {k: v.astype(np.float64) for k, v in sd.items()}
    sm = {k: v.astype(np.float64) for k, v in sd.items()}
    sp["fc.1.weight"] = sp["fc.1.weight"].copy()
    sm["fc.1.weight"] = sm["fc.1.weight"].copy()
    sp["fc.1.weight"][3, 2] += h
    sm["fc.1.weight"][3, 2] -= h
    fd = (f(sp) - f(sm)) / (2 * h)
    assert abs(fd - gr["fc.1.weight"][3, 2]) <= 1e-5 * max(1.0, abs(fd))


def P_nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / nb) if nb > 0 else float(np.linalg.norm(a))
