"""The evaluation-objective restatement (oracle/dladmm_oracle_eval.py)
pinned by fixtures that EXECUTED the reference test scripts' own objective statements
(tests/golden/make_golden_eval.py: test_syn_l1l1_scalar.py:450-604, test_syn_lasso_scalar.py:
446-568) on the scripts' own model class.  CPU only."""
import json
import os

import numpy as np
import pytest

import problems as P
from conftest import GOLDEN


def load_eval(name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    return g, json.loads(str(g["meta"]))


@pytest.mark.parametrize("name", sorted(P.EVAL_FIXTURES))
def test_eval_inputs_regenerate_bit_exact(name):
    g, meta = load_eval(name)
    assert meta["case"] == P.EVAL_FIXTURES[name]
    inp, sd = P.eval_problem(meta["case"])
    for k, v in inp.items():
        assert P.sha256(v) == meta["sha256"][k], k
    for k, v in sd.items():
        assert P.sha256(v) == meta["sha256"]["sd:" + k], k


@pytest.mark.parametrize("name", sorted(P.EVAL_FIXTURES))
def test_eval_restatement_matches_reference_statements(name):
    """Every objective of the restatement, accumulated over the fixture's batches on the
    reference's own forward outputs and finalised like the script, equals what the script's
    statements computed (fp32 accumulators in the reference, fp64 here)."""
    from oracle import dladmm_oracle_eval as oe
    g, meta = load_eval(name)
    c = meta["case"]
    inp, _ = P.eval_problem(c)
    bs, nb, K, alpha = c["batch_size"], c["n_batches"], c["layers"], c["alpha"]
    n_test = bs * nb
    A = inp["A"]
    cols = lambda a, j: a[:, j * bs:(j + 1) * bs]  # noqa: E731
    acc = {}
    for j in range(nb):
        Z, E, L, T = (list(g["ref_" + nm][j]) for nm in "ZELT")
        X = cols(inp["X"], j)
        vals = {}
        if "NMSE" in c["objectives"]:
            vals["NMSE"] = np.stack(oe.nmse_terms(Z, E, cols(inp["Zstar"], j),
                                                  cols(inp["Estar"], j)))
        if "L1L1" in c["objectives"]:
            vals["L1L1"] = oe.l1l1(Z, X, A, alpha)
        if "LASSO" in c["objectives"]:
            vals["LASSO"] = oe.lasso(Z, X, A, alpha)
            vals["LASSO-ALL"] = oe.lasso(Z, X, A, alpha, per_sample=True)
        if c["gt_K"]:
            Zg, Eg = g["gt_Z"][j], g["gt_E"][j]
            vals["Normalized-L1L1"] = oe.normalized_l1l1(Z, X, A, alpha, Zg)
            vals["GT"] = oe.gt(Z, E, Zg, Eg)
            vals["Normalized-GT"] = oe.normalized_gt(Z, E, Zg, Eg)
            Lc = np.float32(np.linalg.norm(A.T @ A, ord=2))   # test_syn_l1l1_scalar.py:90
            vals["S-L2"] = oe.s_l2(Z, E, L, T, X, A, inp["E0"], alpha, Lc)
        for k, v in vals.items():
            if k == "LASSO-ALL":
                acc.setdefault(k, []).append(v)
            else:
                acc[k] = acc.get(k, 0) + v
    for ob in c["objectives"]:
        ref = g["obj_" + ob]
        if ob == "NMSE":
            dz = (inp["Zstar"].astype(np.float64) ** 2).sum() / n_test
            de = (inp["Estar"].astype(np.float64) ** 2).sum() / n_test
            got = 10 * np.log10(acc[ob][0] / n_test / dz + acc[ob][1] / n_test / de)
            np.testing.assert_allclose(got, ref, atol=1e-5)   # dB: a difference, not a ratio
        elif ob == "LASSO-ALL":
            np.testing.assert_allclose(np.concatenate(acc[ob]), ref, rtol=1e-5)
        else:
            np.testing.assert_allclose(acc[ob] / n_test, ref, rtol=2e-5, err_msg=ob)
        assert ref.shape[-1] == K
