"""Generate the golden fixtures under tests/golden/ from the REFERENCE implementation.

Runs in the build container only (it reads /root/reference).  For each fixture in
problems.FIXTURES it
  1. regenerates the synthetic inputs and the parameter set (problems.build_problem),
  2. takes the reference `class DLADMMNet` of the variant's script *as source text*, parses it
     with `ast` and executes ONLY that class definition (the scripts' module level would parse
     argv, read missing .mat blobs and start training), with `.cuda()` patched to identity,
  3. constructs it with the reference ctor signature, `load_state_dict(strict=True)` the
     parameter set, and runs `forward` on CPU under no_grad in fp32 and in fp64,
  4. computes the per-layer training objectives exactly as the reference training loops do
     (L1L1: main_syn_l1l1_scalar.py:290-294; LASSO: main_syn_lasso_scalar.py:276-281),
  5. writes `<name>.npz` with the outputs, the fp32-vs-fp64 gaps, the state_dict key list and the
     sha256 of every regenerated input array.
It also writes dladmm_v1_layout.pth.tar: a raw state_dict saved by the reference V1 class
(main_lena.py:243 / test_lena_lskm.py:284-285 layout, 45 keys at layers=15).

Usage:  python tests/golden/make_golden.py [--ref /root/reference] [names...]
"""
from __future__ import annotations

import argparse
import ast
import json
import math
import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import problems  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ALPHA = 0.001  # -a default of main_syn_l1l1_scalar.py:21 and alpha of main_syn_lasso_scalar.py:190


def load_ref_cls(path: str, name: str = "DLADMMNet"):
    src = open(path).read()
    for node in ast.parse(src).body:
        if isinstance(node, ast.ClassDef) and node.name == name:
            ns = dict(torch=torch, nn=nn, F=F, np=np, sqrt=math.sqrt)
            exec(compile(ast.Module([node], []), path, "exec"), ns)
            return ns[name]
    raise RuntimeError(f"class {name} not found in {path}")


def run_ref(cls, inp, sd, K, dtype, interval=0, fwd_k=False):
    conv = lambda a: torch.from_numpy(np.asarray(a)).to(dtype)  # noqa: E731
    m, n = inp["A"].shape
    B = inp["X"].shape[1]
    extra = {"interval": interval} if interval else {}
    net = cls(m=m, n=0, d=n, batch_size=B, A=conv(inp["A"]), Z0=conv(inp["Z0"]),
              E0=conv(inp["E0"]), L0=conv(inp["L0"]), layers=K, **extra)
    net.load_state_dict({k: conv(v) for k, v in sd.items()}, strict=True)
    net = net.to(dtype)
    keys = list(net.state_dict().keys())
    with torch.no_grad():
        out = net(conv(inp["X"]), K) if fwd_k else net(conv(inp["X"]))
    return out, keys


def losses(Zs, X, A):
    """Per-layer objectives as the reference training loops compute them."""
    l1l1, lasso = [], []
    for Zk in Zs:
        r = X - torch.mm(A, Zk)
        l1l1.append(float(ALPHA * torch.sum(torch.abs(Zk), dim=0).mean()
                          + torch.sum(torch.abs(r), dim=0).mean()))
        lasso.append(float(ALPHA * torch.sum(torch.abs(Zk), dim=0).mean()
                           + 0.5 * torch.sum(r ** 2.0, dim=0).mean()))
    return np.array(l1l1, np.float64), np.array(lasso, np.float64)


def nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def make_one(name, defn, ref_root):
    # Both patches only matter inside the reference ctor (main_lena.py:23-26 calls .cuda()).
    torch.Tensor.cuda = lambda self, *a, **k: self
    nn.Module.cuda = lambda self, *a, **k: self
    variant = defn["variant"]
    cls = load_ref_cls(os.path.join(ref_root, problems.VARIANT_SOURCES[variant]))
    inp, sd = problems.build_problem(defn)
    K = defn["K"]
    spec = problems.VARIANT_SPECS[variant]
    kw = dict(interval=defn.get("interval", 0), fwd_k=spec.get("fwd_k", False))
    out32, keys = run_ref(cls, inp, sd, K, torch.float32, **kw)
    out64, _ = run_ref(cls, inp, sd, K, torch.float64, **kw)
    names = ["Z", "E", "L", "T"][: len(out32)]
    rec = {}
    for nm, seq32, seq64 in zip(names, out32, out64):
        a32 = np.stack([t.numpy() for t in seq32]).astype(np.float32)
        a64 = np.stack([t.numpy() for t in seq64])
        rec[nm] = a32
        rec["gap_" + nm] = np.array([nrel(a32[k], a64[k]) for k in range(a32.shape[0])])
    A32 = torch.from_numpy(inp["A"])
    X32 = torch.from_numpy(inp["X"])
    rec["loss_l1l1"], rec["loss_lasso"] = losses(out32[0], X32, A32)
    shas = {k: problems.sha256(v) for k, v in inp.items()}
    shas.update({"sd:" + k: problems.sha256(v) for k, v in sd.items()})
    rec["meta"] = np.array(json.dumps(dict(name=name, defn=defn, keys=keys, sha256=shas,
                                           alpha=ALPHA, torch=torch.__version__,
                                           source=problems.VARIANT_SOURCES[variant])))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **rec)
    gaps = {k: float(np.max(v)) for k, v in rec.items() if k.startswith("gap_")}
    print(f"{name:22s} keys={len(keys):4d} {os.path.getsize(path)/1e6:6.2f} MB  max fp32-vs-fp64 gap {gaps}")


def make_layout(ref_root):
    torch.Tensor.cuda = lambda self, *a, **k: self
    nn.Module.cuda = lambda self, *a, **k: self
    cls = load_ref_cls(os.path.join(ref_root, "main_lena.py"))
    m, n, B, K = 16, 32, 20, 15
    inp = problems.make_inputs(m, n, B, 4242)
    torch.manual_seed(4242)
    net = cls(m=m, n=0, d=n, batch_size=B, A=torch.from_numpy(inp["A"]),
              Z0=torch.from_numpy(inp["Z0"]), E0=torch.from_numpy(inp["E0"]),
              L0=torch.from_numpy(inp["L0"]), layers=K)
    sd = net.state_dict()
    path = os.path.join(HERE, "dladmm_v1_layout.pth.tar")
    torch.save(sd, path)
    print(f"layout: {len(sd)} keys -> {path}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    torch.set_num_threads(8)
    names = a.names or list(problems.FIXTURES)
    for nm in names:
        make_one(nm, problems.FIXTURES[nm], a.ref)
    if not a.names:
        make_layout(a.ref)


if __name__ == "__main__":
    main()
