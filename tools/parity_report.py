"""Per-layer error report of the HIP forward on every golden fixture (GPU box diagnostic).

For each output and layer prints nrel(hip, ref32), nrel(hip, oracle64) and the reference's own
gap nrel(ref32, ref64): a kernel as accurate as the reference has nrel(hip, oracle64) ~ gap.
    python tools/parity_report.py [fixture ...]
"""
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import problems as P  # noqa: E402
from conftest import load_golden  # noqa: E402
from oracle import dladmm_oracle as O  # noqa: E402
from test_gpu_parity import make_net, nrel  # noqa: E402


def main(names):
    dl = importlib.import_module("d-ladmm_amd")
    worst = 0.0
    for name in names or sorted(P.FIXTURES):
        g, meta = load_golden(name)
        d = meta["defn"]
        inp, sd = P.build_problem(d)
        net = make_net(dl, d["variant"], inp, sd, d["K"])
        with torch.no_grad():
            out = net(torch.from_numpy(inp["X"]).cuda())
        ref64 = O.forward(d["variant"], inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd,
                          d["K"], dtype=np.float64)
        for nm, seq in zip(["Z", "E", "L", "T"], out):
            if nm not in g.files:
                continue
            for k, t in enumerate(seq):
                got = t.cpu().numpy()
                e32 = nrel(got, g[nm][k])
                r64 = ref64[nm if nm != "T" or "T" in ref64 else "T_internal"][k]
                e64 = nrel(got, r64)
                gap = float(g["gap_" + nm][k])
                ratio = e64 / max(gap, 1e-12)
                worst = max(worst, ratio if gap > 1e-7 else 0.0)
                print(f"{name:14s} {nm}[{k:2d}]  vs ref32 {e32:.2e}  vs f64 {e64:.2e}  "
                      f"ref gap {gap:.2e}  (f64 err / gap {ratio:5.2f})")
    print(f"worst (hip vs f64) / (ref32 vs f64) over layers with gap > 1e-7: {worst:.2f}")


if __name__ == "__main__":
    main(sys.argv[1:])
