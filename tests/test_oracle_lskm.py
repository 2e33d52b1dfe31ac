"""The classic KM / LSKM oracle (oracle/dladmm_oracle_lskm.py) is pinned against the reference
test-script class run on the same inputs (tests/golden/make_golden_lskm.py).  CPU only."""
import numpy as np
import pytest

from conftest import load_golden
import problems as P


def nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def run_case(case):
    from oracle import dladmm_oracle_lskm as ol
    inp, sd = P.build_problem(case["defn"])
    return ol.lskm_forward(inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd,
                           case["layers"], case["learned"], case["safeguard"], case["continued"],
                           case["K"], case["alpha"], case["delta"], case["mu"], case["mu_param"])


@pytest.mark.parametrize("name", sorted(P.LSKM_FIXTURES))
def test_lskm_oracle_matches_reference(name):
    g, meta = load_golden(name)
    case = meta["case"]
    assert case == P.LSKM_FIXTURES[name]
    out = run_case(case)
    pick = list(g["layers_kept"])
    for nm in ("Z", "E", "L", "T"):
        seq = out[nm]
        got = [seq[j + 1] if nm == "T" else seq[j] for j in pick]
        for i, j in enumerate(pick):
            tol = max(1e-5, 3.0 * float(g["gap_" + nm][i]))
            assert nrel(got[i], g[nm][i]) <= tol, (nm, j)
    if "sg_count" in g.files:
        np.testing.assert_array_equal(out["sg_count"], g["sg_count"])
