"""The dual-gap objective checker (tests/lena_checker.py over the torch-op restatement
oracle/dladmm_torch_cpu.py) against the reference scripts' own loss statements, executed on their
own model classes (tests/golden/lena_*.npz, make_golden_lena.py): main_lena.py:221-231 and
main_syn_l1l1-dgap_ltheta.py:196-211 (minus sign, last layer only).  CPU only.  The same ATen ops
in the same order on the same torch build: the fp32 loss values and gradients agree with the
reference's fp32 run to rounding (1e-6 norm-relative), well inside the GPU tests' bars."""
import numpy as np
import pytest
import torch

from conftest import load_golden
import problems as P
from lena_checker import lena_losses
from oracle import dladmm_torch_cpu as tcpu


def nrel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / nb) if nb > 0 else float(np.linalg.norm(a))


@pytest.mark.parametrize("name", sorted(P.LENA_FIXTURES))
def test_lena_checker_matches_reference_statements(name):
    g, meta = load_golden(name)
    d = meta["defn"]
    assert d == P.LENA_FIXTURES[name]["defn"]
    inp, sd = P.build_problem(d)
    K = d["K"]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    params = {k: t(v).clone().requires_grad_(True) for k, v in sd.items()}
    X, A = t(inp["X"]), t(inp["A"])
    fwd = getattr(tcpu.forward, "__wrapped__", tcpu.forward)
    with torch.enable_grad():
        out = fwd(d["variant"], X, A, t(inp["Z0"]), t(inp["E0"]), t(inp["L0"]), params, K)
        per = lena_losses(out[0], out[1], out[2], X, A, meta["alpha"], K, meta["lx_sign"],
                          meta["loss_start_layer"])
        total = sum(per)
        total.backward()
    t32, t64 = g["total"]
    assert abs(float(total) - t32) <= 1e-6 * abs(t64)
    per_ref = g["per_layer"][0]
    assert nrel([float(v) for v in per], per_ref) <= 1e-6
    for k in sd:
        ref = g["g:" + k]
        mine = params[k].grad
        mine = np.zeros_like(ref) if mine is None else mine.numpy()
        assert nrel(mine, ref) <= max(1e-6, float(g["gap:" + k])), k
