"""The torch-op CPU restatement (oracle/dladmm_torch_cpu.py: bench.py's CPU baseline) is pinned to
the golden fixtures the reference classes produced (tests/golden/make_golden.py).  It issues the
reference's own ATen ops in the reference's order on the same torch build, so it reproduces the
fixtures bit for bit.  CPU only."""
import numpy as np
import pytest
import torch

from conftest import load_golden
import problems as P
from oracle import dladmm_torch_cpu as tcpu

NAMES = sorted(n for n in P.FIXTURES
               if load_golden(n)[1]["defn"]["variant"] in ("v1", "v2", "v3", "v4", "v5", "v6"))


@pytest.mark.parametrize("name", NAMES)
def test_torch_restatement_matches_reference(name):
    g, meta = load_golden(name)
    d = meta["defn"]
    inp, sd = P.build_problem(d)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    out = tcpu.forward(d["variant"], t(inp["X"]), t(inp["A"]), t(inp["Z0"]), t(inp["E0"]),
                       t(inp["L0"]), {k: t(v) for k, v in sd.items()}, d["K"])
    names = "ZELT"[:len(out)]
    assert ("T" in g.files) == (len(out) == 4)
    for nm, seq in zip(names, out):
        ref = g[nm]
        assert len(seq) == ref.shape[0]
        for k in range(ref.shape[0]):
            np.testing.assert_array_equal(seq[k].numpy(), ref[k], err_msg=f"{name} {nm}[{k}]")
