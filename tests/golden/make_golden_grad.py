"""Generate the gradient fixtures tests/golden/grad_*.npz from the REFERENCE implementation.

Build container only (reads /root/reference).  For each entry of problems.GRAD_FIXTURES:
  1. regenerate the base forward fixture's inputs and parameters (problems.build_problem) and the
     seeded upstream cotangents (problems.make_upstream),
  2. take the reference `class DLADMMNet` as source text and execute only that class (as
     make_golden.py does), construct it, `load_state_dict(strict=True)` the parameters,
  3. run forward with autograd on CPU, build the loss of problems.GRAD_FIXTURES (the reference
     training loss + the random linear terms), call `.backward()` -- the reference's own
     training-step mechanism (main_syn_l1l1_scalar.py:298) -- in fp32 and in fp64,
  4. write every parameter's .grad (state_dict key names), the fp32-vs-fp64 gap per key, the loss
     value and the sha256 of the regenerated cotangents.

Usage:  python tests/golden/make_golden_grad.py [--ref /root/reference] [names...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import problems  # noqa: E402
from make_golden import load_ref_cls, nrel  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def run_grad(cls, inp, sd, up, K, kind, dtype, interval=0, fwd_k=False):
    conv = lambda a: torch.from_numpy(np.asarray(a)).to(dtype)  # noqa: E731
    m, n = inp["A"].shape
    B = inp["X"].shape[1]
    extra = {"interval": interval} if interval else {}
    net = cls(m=m, n=0, d=n, batch_size=B, A=conv(inp["A"]), Z0=conv(inp["Z0"]),
              E0=conv(inp["E0"]), L0=conv(inp["L0"]), layers=K, **extra)
    net.load_state_dict({k: conv(v) for k, v in sd.items()}, strict=True)
    net = net.to(dtype)
    X = conv(inp["X"])
    A = conv(inp["A"])
    out = net(X, K) if fwd_k else net(X)
    Z, E, L = out[0], out[1], out[2]
    coeffs = problems.loss_coeffs(K)
    total = 0
    alpha = problems.GRAD_ALPHA
    for k in range(K):  # main_syn_l1l1_scalar.py:283-296 / main_syn_lasso_scalar.py:270-283
        if kind == "l1l1":
            lk = alpha * torch.sum(torch.abs(Z[k]), dim=0).mean() + \
                torch.sum(torch.abs(X - torch.mm(A, Z[k])), dim=0).mean()
        else:
            lk = alpha * torch.sum(torch.abs(Z[k]), dim=0).mean() + \
                0.5 * torch.sum((X - torch.mm(A, Z[k])) ** 2.0, dim=0).mean()
        total = total + lk * coeffs[k]
    for k in range(K if up is not None else 0):
        # newS: E[0] / L[0] are the inputs E0 / L0 (no parameter reaches them)
        total = total + (conv(up["Gz"][k]) * Z[k]).sum() + (conv(up["Ge"][k]) * E[k]).sum() + \
            (conv(up["Gl"][k]) * L[k]).sum()
    if up is not None and "Gt" in up:
        T = out[3]
        for j in range(K + 1):
            total = total + (conv(up["Gt"][j]) * T[j]).sum()
    total.backward()
    grads = {k: (p.grad.detach().numpy().copy() if p.grad is not None
                 else np.zeros(tuple(p.shape))) for k, p in net.named_parameters()}
    run_grad.none_keys = [k for k, p in net.named_parameters() if p.grad is None]
    return grads, float(total.detach())


def make_one(name, gdef, ref_root):
    torch.Tensor.cuda = lambda self, *a, **k: self
    nn.Module.cuda = lambda self, *a, **k: self
    defn = problems.grad_defn(gdef)
    variant = defn["variant"]
    cls = load_ref_cls(os.path.join(ref_root, problems.VARIANT_SOURCES[variant]))
    inp, sd = problems.build_problem(defn)
    ret_t = problems.VARIANT_SPECS[variant]["ret_t"]
    up = problems.make_upstream(defn, ret_t)
    kw = dict(interval=defn.get("interval", 0),
              fwd_k=problems.VARIANT_SPECS[variant].get("fwd_k", False))
    g32, l32 = run_grad(cls, inp, sd, up, defn["K"], gdef["loss"], torch.float32, **kw)
    g64, l64 = run_grad(cls, inp, sd, up, defn["K"], gdef["loss"], torch.float64, **kw)
    rec = {}
    for k in sd:
        rec["g:" + k] = g32[k].astype(np.float32)
        rec["gap:" + k] = np.array(nrel(g32[k], g64[k]))
    rec["loss"] = np.array([l32, l64])
    shas = {k: problems.sha256(v) for k, v in up.items()}
    rec["meta"] = np.array(json.dumps(dict(name=name, gdef=gdef, defn=defn, keys=list(sd.keys()),
                                           sha256=shas, alpha=problems.GRAD_ALPHA,
                                           coeffs=problems.loss_coeffs(defn["K"]),
                                           torch=torch.__version__,
                                           source=problems.VARIANT_SOURCES[variant])))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **rec)
    worst = max(float(rec["gap:" + k]) for k in sd)
    print(f"{name:20s} keys={len(sd):4d} {os.path.getsize(path)/1e6:6.2f} MB  "
          f"max fp32-vs-fp64 grad gap {worst:.2e}")


def make_none_keys(ref_root):
    """tests/golden/grad_none_keys.json: the parameters whose .grad the REFERENCE autograd
    leaves None (outside the loss graph; the .npz fixtures store zeros for them), for every
    gradient fixture's loss and for the bare training loss (Z terms only, no linear terms)."""
    torch.Tensor.cuda = lambda self, *a, **k: self
    nn.Module.cuda = lambda self, *a, **k: self
    out = {}
    for name, gdef in problems.GRAD_FIXTURES.items():
        defn = problems.grad_defn(gdef)
        variant = defn["variant"]
        cls = load_ref_cls(os.path.join(ref_root, problems.VARIANT_SOURCES[variant]))
        inp, sd = problems.build_problem(defn)
        up = problems.make_upstream(defn, problems.VARIANT_SPECS[variant]["ret_t"])
        kw = dict(interval=defn.get("interval", 0),
                  fwd_k=problems.VARIANT_SPECS[variant].get("fwd_k", False))
        rec = {}
        for tag, u in (("fixture_loss", up), ("training_loss", None)):
            run_grad(cls, inp, sd, u, defn["K"], gdef["loss"], torch.float32, **kw)
            rec[tag] = run_grad.none_keys
        out[name] = rec
        print(name, rec)
    with open(os.path.join(HERE, "grad_none_keys.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--none-keys", action="store_true")
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    torch.set_num_threads(8)
    if a.none_keys:
        make_none_keys(a.ref)
        return
    for nm in a.names or list(problems.GRAD_FIXTURES):
        make_one(nm, problems.GRAD_FIXTURES[nm], a.ref)


if __name__ == "__main__":
    main()
