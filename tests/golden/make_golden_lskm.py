"""Generate tests/golden/lskm_*.npz from the REFERENCE test-script class (SURVEY.md section 8
row f2: classic KM / learned + safeguarded KM).

Build container only (reads /root/reference).  The class `DLADMMNet` of
test_syn_l1l1_scalar.py:73-322 reads module globals (alpha, delta, mu_k_method, mu_k_param,
mu_updater_dict, args.continued, K), so only that class definition -- parsed with `ast` -- and
the updater classes of mu_updater.py are executed, in a namespace that supplies those globals;
the script's module level (argparse, .mat loading, testing loop) never runs.  For each case the
class is constructed with the reference ctor, the V4 parameter set is loaded with
load_state_dict(strict=True) and forward(x, use_learned, use_safeguard, continued, K) runs on
CPU in fp32 and fp64.  Stored: Z/E/L/T at selected layers, sg_count, fp32-vs-fp64 gaps.

Usage:  python tests/golden/make_golden_lskm.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import ast
import json
import math
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import problems  # noqa: E402
from make_golden import nrel  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def load_classes(path, names, ns):
    for node in ast.parse(open(path).read()).body:
        if isinstance(node, ast.ClassDef) and node.name in names:
            exec(compile(ast.Module([node], []), path, "exec"), ns)


def ref_class(ref_root, case, dtype):
    ns = dict(torch=torch, nn=nn, F=F, np=np, sqrt=math.sqrt)
    load_classes(os.path.join(ref_root, "mu_updater.py"),
                 {"EMAUpdater", "GSUpdater", "RTUpdater", "RMUpdater", "BlankUpdater"}, ns)
    ns["mu_updater_dict"] = {"EMA": ns["EMAUpdater"], "GS": ns["GSUpdater"],
                             "RT": ns["RTUpdater"], "RM": ns["RMUpdater"],
                             "None": ns["BlankUpdater"]}
    ns.update(alpha=case["alpha"], delta=case["delta"], mu_k_method=case["mu"],
              mu_k_param=case["mu_param"], layers=case["layers"], K=case["K"],
              args=types.SimpleNamespace(continued=case["continued"]))
    load_classes(os.path.join(ref_root, "test_syn_l1l1_scalar.py"), {"DLADMMNet"}, ns)
    return ns["DLADMMNet"]


def run(ref_root, case, dtype):
    torch.Tensor.cuda = lambda self, *a, **k: self
    nn.Module.cuda = lambda self, *a, **k: self
    d = case["defn"]
    inp, sd = problems.build_problem(d)
    cls = ref_class(ref_root, case, dtype)
    conv = lambda a: torch.from_numpy(np.asarray(a)).to(dtype)  # noqa: E731
    m, n = inp["A"].shape
    B = inp["X"].shape[1]
    net = cls(m=m, n=0, d=n, batch_size=B, A=conv(inp["A"]), Z0=conv(inp["Z0"]),
              E0=conv(inp["E0"]), L0=conv(inp["L0"]), layers=case["layers"])
    net.load_state_dict({k: conv(v) for k, v in sd.items()}, strict=True)
    net = net.to(dtype)
    net.L = net.L.to(dtype)
    with torch.no_grad():
        out = net(conv(inp["X"]), case["learned"], case["safeguard"], case["continued"],
                  K=case["K"])
    return out, list(net.state_dict().keys())


def make_one(name, case, ref_root):
    o32, keys = run(ref_root, case, torch.float32)
    o64, _ = run(ref_root, case, torch.float64)
    K = case["K"]
    pick = sorted({0, 1, K // 2, K - 1})
    rec = {"layers_kept": np.array(pick)}
    for i, nm in enumerate(("Z", "E", "L", "T")):
        a32, a64 = o32[i], o64[i]
        idx = pick if nm != "T" else [j + 1 for j in pick]  # T[0] = A Z0 + E0 - X
        rec[nm] = np.stack([a32[j].numpy() for j in idx]).astype(np.float32)
        rec["gap_" + nm] = np.array([nrel(a32[j].numpy(), a64[j].numpy()) for j in idx])
    if len(o32) == 5:
        rec["sg_count"] = np.asarray(o32[4], np.float64)
        rec["sg_count64"] = np.asarray(o64[4], np.float64)
    rec["meta"] = np.array(json.dumps(dict(name=name, case=case, keys=keys,
                                           torch=torch.__version__,
                                           source="test_syn_l1l1_scalar.py")))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **rec)
    sg = rec.get("sg_count")
    print(f"{name:24s} {os.path.getsize(path)/1e3:7.1f} kB  max gap "
          f"{max(float(np.max(rec['gap_' + k])) for k in 'ZELT'):.2e}  sg_count "
          f"{None if sg is None else sg.tolist()}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    torch.set_num_threads(8)
    for nm in a.names or list(problems.LSKM_FIXTURES):
        make_one(nm, problems.LSKM_FIXTURES[nm], a.ref)


if __name__ == "__main__":
    main()
