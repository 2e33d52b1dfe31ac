"""Debug helper: run small problems through the forced per-layer path and report per-output
errors against the oracle (run on the GPU box)."""
import importlib, os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import problems as P
from oracle import dladmm_oracle as O
os.environ["DLADMM_PATH"] = "layered"
dl = importlib.import_module("d-ladmm_amd")
for (m, n, B, K) in [(16, 32, 16, 1), (32, 256, 128, 1), (256, 512, 128, 1), (300, 600, 150, 2)]:
    inp = P.make_inputs(m, n, B, 1)
    sd = P.make_state_dict("v4", m, n, B, K, inp["A"], 1, perturb=0.1)
    t = torch.from_numpy
    net = dl.DLADMMNetScalar(m=m, n=0, d=n, batch_size=B, A=t(inp["A"]), Z0=t(inp["Z0"]),
                             E0=t(inp["E0"]), L0=t(inp["L0"]), layers=K)
    net.load_state_dict({k: t(v) for k, v in sd.items()}); net.requires_grad_(False)
    with torch.no_grad():
        Z, E, L, T = net(t(inp["X"]).cuda())
    ref = O.forward("v4", inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, K)
    T0 = inp["A"] @ inp["Z0"] + inp["E0"] - inp["X"]
    print((m, n, B, K), "T0", O.nrel(T[0].cpu().numpy(), T0),
          "Z0", O.nrel(Z[0].cpu().numpy(), ref["Z"][0]),
          "E0", O.nrel(E[0].cpu().numpy(), ref["E"][0]), "T1", O.nrel(T[1].cpu().numpy(), ref["T"][1]))
    z = Z[0].cpu().numpy(); r = ref["Z"][0]
    bad = np.argwhere(np.abs(z - r) > 1e-3 * (1 + np.abs(r)))
    print("  bad rows", np.unique(bad[:, 0])[:20], "bad cols", np.unique(bad[:, 1])[:20], len(bad))
