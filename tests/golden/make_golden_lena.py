"""Generate tests/golden/lena_*.npz: the dual-gap training objective of the REFERENCE scripts.

Build container only (reads /root/reference).  For each problems.LENA_FIXTURES entry:
  1. regenerate the forward problem (problems.build_problem);
  2. take from the script's source text, with `ast`, and execute ONLY:
       - its `class DLADMMNet` (as make_golden.py does),
       - its `def dual_gap` (main_lena.py:145-147; main_syn_l1l1-dgap_ltheta.py:118-120),
       - its module-level `alpha = ...` and (dgap script) `loss_start_layer = layers - 1`,
       - the training step's loss loop: the `for k in range(layers):` statement whose body
         appends to `loss` (main_lena.py:221-231; main_syn_l1l1-dgap_ltheta.py:196-209),
     with the script's own variable names bound: Z, E, L from the model's forward, A_tensor,
     input_bs_var = X, layers = K, loss = list(), total_loss = 0;
  3. call `total_loss.backward()` -- the script's next statement -- in fp32 and in fp64;
  4. write total_loss, the per-layer `loss` list, every parameter's .grad (state_dict names) and
     the fp32-vs-fp64 gaps.
The script's module level (argv, .mat loads, the training loop around the statement) never runs.

Usage:  python tests/golden/make_golden_lena.py [--ref /root/reference] [names...]
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
from make_golden import load_ref_cls, nrel  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def _is_loss_loop(node) -> bool:
    """`for k in range(layers): ... loss.append(...)` -- the training step's loss loop."""
    if not (isinstance(node, ast.For) and isinstance(node.target, ast.Name) and
            node.target.id == "k" and isinstance(node.iter, ast.Call) and
            getattr(node.iter.func, "id", None) == "range" and
            [getattr(a, "id", None) for a in node.iter.args] == ["layers"]):
        return False
    for sub in ast.walk(node):
        if isinstance(sub, ast.Call) and isinstance(sub.func, ast.Attribute) and \
                sub.func.attr == "append" and getattr(sub.func.value, "id", None) == "loss":
            return True
    return False


def extract(path: str):
    """(dual_gap FunctionDef, module-level Assign nodes of alpha / loss_start_layer, the loss
    loop For node) from the script's source text."""
    tree = ast.parse(open(path).read())
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "dual_gap")
    assigns = [n for n in tree.body if isinstance(n, ast.Assign) and len(n.targets) == 1 and
               getattr(n.targets[0], "id", None) in ("alpha", "loss_start_layer")]
    loops = [n for n in ast.walk(tree) if _is_loss_loop(n)]
    if not loops:
        raise RuntimeError(f"no training loss loop in {path}")
    return fn, assigns, loops[0]


def lx_sign_of(loop) -> float:
    """Sign with which the loop adds the mean(L[k] * input_bs_var) term: the BinOp whose right
    operand reads input_bs_var (recorded for the tests, which pass it to training_loss)."""
    for sub in ast.walk(loop):
        if isinstance(sub, ast.BinOp) and any(
                isinstance(x, ast.Name) and x.id == "input_bs_var" for x in ast.walk(sub.right)):
            return -1.0 if isinstance(sub.op, ast.Sub) else 1.0
    raise RuntimeError("no L * X term in the loss loop")


def run_lena(cls, stmts, inp, sd, K, dtype, path):
    conv = lambda a: torch.from_numpy(np.asarray(a)).to(dtype)  # noqa: E731
    m, n = inp["A"].shape
    B = inp["X"].shape[1]
    net = cls(m=m, n=0, d=n, batch_size=B, A=conv(inp["A"]), Z0=conv(inp["Z0"]),
              E0=conv(inp["E0"]), L0=conv(inp["L0"]), layers=K)
    net.load_state_dict({k: conv(v) for k, v in sd.items()}, strict=True)
    net = net.to(dtype)
    X = conv(inp["X"])
    out = net(X)
    fn, assigns, loop = stmts
    ns = dict(torch=torch, F=F, nn=nn, np=np, sqrt=math.sqrt, layers=K)
    exec(compile(ast.Module([fn] + assigns, []), path, "exec"), ns)
    ns.update(Z=out[0], E=out[1], L=out[2], A_tensor=conv(inp["A"]), input_bs_var=X,
              loss=list(), total_loss=0)
    exec(compile(ast.Module([loop], []), path, "exec"), ns)
    total = ns["total_loss"]
    total.backward()
    grads = {k: (p.grad.detach().numpy().copy() if p.grad is not None
                 else np.zeros(tuple(p.shape))) for k, p in net.named_parameters()}
    per = [float(v.detach()) if torch.is_tensor(v) else float(v) for v in ns["loss"]]
    return grads, float(total.detach()), per, ns["alpha"], ns.get("loss_start_layer", 0)


def make_one(name, fx, ref_root):
    torch.Tensor.cuda = lambda self, *a, **k: self
    nn.Module.cuda = lambda self, *a, **k: self
    defn = fx["defn"]
    path = os.path.join(ref_root, fx["script"])
    cls = load_ref_cls(path)
    stmts = extract(path)
    inp, sd = problems.build_problem(defn)
    g32, t32, p32, alpha, start = run_lena(cls, stmts, inp, sd, defn["K"], torch.float32, path)
    g64, t64, p64, _, _ = run_lena(cls, stmts, inp, sd, defn["K"], torch.float64, path)
    rec = {}
    for k in sd:
        rec["g:" + k] = g32[k].astype(np.float32)
        rec["gap:" + k] = np.array(nrel(g32[k], g64[k]))
    rec["total"] = np.array([t32, t64])
    rec["per_layer"] = np.array([p32, p64])
    lx_sign = lx_sign_of(stmts[2])
    meta = dict(name=name, defn=defn, script=fx["script"], keys=list(sd.keys()), alpha=alpha,
                loss_start_layer=start, lx_sign=lx_sign,
                loop_lines=[stmts[2].lineno, stmts[2].end_lineno],
                dual_gap_lines=[stmts[0].lineno, stmts[0].end_lineno], torch=torch.__version__)
    rec["meta"] = np.array(json.dumps(meta))
    out = os.path.join(HERE, name + ".npz")
    np.savez_compressed(out, **rec)
    worst = max(float(rec["gap:" + k]) for k in sd)
    print(f"{name:16s} {fx['script']:32s} alpha={alpha} start={start} lx_sign={lx_sign:+.0f} "
          f"total {t32:.7g} / {t64:.7g}  max grad gap {worst:.2e}  "
          f"{os.path.getsize(out) / 1e6:.2f} MB")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    torch.set_num_threads(8)
    for nm in a.names or list(problems.LENA_FIXTURES):
        make_one(nm, problems.LENA_FIXTURES[nm], a.ref)


if __name__ == "__main__":
    main()
