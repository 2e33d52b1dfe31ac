"""Quick check of path 6 (dladmm_fused_xs.hip) against path 1 at B = 20 / 300, V4 K = 6: bit
equality of every output and the wall time of each call (a hand-off that never completes shows
up as seconds per call, never a hang: every poll is bounded)."""
import importlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import problems as P  # noqa: E402


def main():
    dl = importlib.import_module("d-ladmm_amd")
    ops, L = dl.ops, dl._lib
    for B in (20, 300):
        d = dict(variant="v4", m=250, n=500, B=B, K=6, seed=77 + B, perturb=0.2, wscale=0.4)
        inp, sd = P.build_problem(d)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
        net = dl.VARIANTS["v4"](m=250, n=0, d=500, batch_size=B, A=t(inp["A"]), Z0=t(inp["Z0"]),
                                E0=t(inp["E0"]), L0=t(inp["L0"]), layers=6)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
        net.cuda().requires_grad_(False)
        X = t(inp["X"])
        tab = net._tables(X.device)
        W = [w.detach() for w in net._weights()]
        out = {}
        for fl in (0, L.F_NO_XSPLIT, L.F_NO_ROWSPLIT):
            torch.cuda.synchronize()
            t0 = time.time()
            r = ops.dladmm_forward(net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0,
                                   keep_all=True, want_T=True, flags=fl, **tab)
            torch.cuda.synchronize()
            out[fl] = (r, time.time() - t0)
            print(f"B={B} flags={fl} path={r.path} wall={out[fl][1] * 1e3:.2f} ms", flush=True)
        for fl in (0, L.F_NO_XSPLIT):
            for nm in ("Z", "E", "L", "T"):
                a, b = getattr(out[fl][0], nm), getattr(out[L.F_NO_ROWSPLIT][0], nm)
                print(f"  flags={fl} {nm} equal={torch.equal(a, b)} "
                      f"maxdiff={float((a - b).abs().max()):.3g}", flush=True)


if __name__ == "__main__":
    main()
