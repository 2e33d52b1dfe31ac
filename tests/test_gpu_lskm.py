"""Classic KM / learned + safeguarded KM on the HIP kernels against
the reference test-script class (golden fixtures, tests/golden/make_golden_lskm.py) and the
oracle (oracle/dladmm_oracle_lskm.py) at the K = 2000 ground-truth depth."""
import numpy as np
import pytest
import torch

from conftest import load_golden
import parity
import problems as P

pytestmark = pytest.mark.gpu


def nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def make(dl, case, inp, sd):
    m, n = inp["A"].shape
    B = inp["X"].shape[1]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    net = dl.DLADMMNetLSKM(m=m, n=0, d=n, batch_size=B, A=t(inp["A"]), Z0=t(inp["Z0"]),
                           E0=t(inp["E0"]), L0=t(inp["L0"]), layers=case["layers"],
                           alpha=case["alpha"], delta=case["delta"], mu_k_method=case["mu"],
                           mu_k_param=case["mu_param"])
    net.load_state_dict({k: t(v) for k, v in sd.items()}, strict=True)
    return net


@pytest.mark.parametrize("name", sorted(P.LSKM_FIXTURES))
def test_lskm_matches_reference(name, dl):
    g, meta = load_golden(name)
    case = meta["case"]
    inp, sd = P.build_problem(case["defn"])
    net = make(dl, case, inp, sd)
    X = torch.from_numpy(inp["X"]).cuda()
    out = net(X, case["learned"], case["safeguard"], case["continued"], K=case["K"])
    assert len(out) == (5 if case["learned"] and case["safeguard"] else 4)
    K = case["K"]
    assert len(out[0]) == K and len(out[3]) == K + 1
    for i, j in enumerate(g["layers_kept"]):
        for c, nm in enumerate("ZELT"):
            got = out[c][j + 1 if nm == "T" else j].cpu().numpy()
            gap = float(g["gap_" + nm][i])
            parity.check(name, "f32", f"{nm}[{int(j)}]", nrel(got, g[nm][i]), parity.tol(gap), gap)
    if "sg_count" in g.files:
        np.testing.assert_array_equal(out[4], g["sg_count"])


def test_km_ground_truth_depth(dl):
    """K = 2000 KM iterations (the test scripts' ground truth, test_syn_l1l1_scalar.py:478) in
    one launch with the weight A^T packed once, against the oracle."""
    from oracle import dladmm_oracle_lskm as ol
    d = dict(variant="v4", m=64, n=128, B=40, K=3, seed=1160, perturb=0.1)
    inp, sd = P.build_problem(d)
    case = dict(layers=3, alpha=0.01, delta=-99.0, mu="None", mu_param=0.0)
    net = make(dl, case, inp, sd)
    X = torch.from_numpy(inp["X"]).cuda()
    Z, E, L, T = net(X, False, False, False, K=2000)
    ref = ol.lskm_forward(inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, 3, False,
                          False, False, 2000, 0.01)
    for k in (0, 9, 99, 1999):
        assert nrel(Z[k].cpu().numpy(), ref["Z"][k]) <= 1e-4, k
        assert nrel(E[k].cpu().numpy(), ref["E"][k]) <= 1e-4, k


@pytest.mark.parametrize("B", [300, 1037])
def test_safeguard_many_columns(B, dl):
    """The safeguard kernel's workgroups of 16 columns x 16 row lanes (row sums in a fixed lane
    order) over many workgroups and a ragged last one, at the test script's m = 250, n = 500:
    safeguard counts and the selected outputs against the oracle's safeguarded forward."""
    from oracle import dladmm_oracle_lskm as ol
    d = dict(variant="v4", m=250, n=500, B=B, K=5, seed=1190 + B, perturb=0.2, wscale=0.9)
    inp, sd = P.build_problem(d)
    case = dict(layers=5, alpha=0.01, delta=0.05, mu="EMA", mu_param=0.5)
    net = make(dl, case, inp, sd)
    X = torch.from_numpy(inp["X"]).cuda()
    Z, E, L, T, cnt = net(X, True, True, False)
    ref = ol.lskm_forward(inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, 5, True,
                          True, False, 5, 0.01, delta=0.05, mu_method="EMA", mu_param=0.5)
    np.testing.assert_array_equal(cnt, ref["sg_count"])
    assert 0 < ref["sg_count"].sum() < 5 * B   # both branches taken
    for k in range(5):
        assert nrel(Z[k].cpu().numpy(), ref["Z"][k]) <= 1e-5, k
        assert nrel(E[k].cpu().numpy(), ref["E"][k]) <= 1e-5, k
        assert nrel(T[k + 1].cpu().numpy(), ref["T"][k + 1]) <= 1e-5, k
