"""Generate tests/golden/eval_*.npz by EXECUTING the reference test scripts' objective code
(NMSE, L1L1, Normalized-L1L1, GT, Normalized-GT, S-L2, LASSO,
LASSO-ALL).

Build container only (reads /root/reference).  The reference computes its evaluation objectives as
inline module-level statements of its test scripts, so there is no function to call.  This script
parses the script as text with `ast` and takes three of its top-level statements:

  * the accumulator set-up `if objective == 'NMSE': mse_z = torch.zeros(K).cuda() ...`
      test_syn_l1l1_scalar.py:450-464, test_syn_lasso_scalar.py:446-458
  * the per-layer accumulation `for jj in range(K): ...` nested in the batch loop
      test_syn_l1l1_scalar.py:483-534, test_syn_lasso_scalar.py:475-505
  * the finalisation `if objective == 'NMSE': ... nmse = 10 * torch.log10(...)`
      test_syn_l1l1_scalar.py:537-604, test_syn_lasso_scalar.py:508-568

and executes exactly those statements (no other line of the script's module level: it would parse
argv, load missing .mat blobs and log to files) in a namespace holding what the script's own batch
loop would hold at that point: the batch `input_bs_var`, the model's forward lists Z, E, L, T of the
batch, the long-KM ground truth (Zp, Ep, Lp, Tp; K = 2000 as at :478), the label batches, the
model (the test script's own `class DLADMMNet`, whose S / two_norm the S-L2 branch calls), alpha.
`.cuda()` is patched to identity and `print` is silenced.  The model is the test script's class
(ast-extracted like make_golden_lskm.py) running use_learned=True, use_safeguard=False on the V4
(l1l1 script) / V6 (lasso script) parameter set of the case.

Stored per case: the finalised per-layer values of every objective (the reference's fp32
accumulators), the reference forward outputs and ground truth per batch (so a test can check the
objective computation alone, on identical inputs), and the sha256 of every regenerated input.

Usage:  python tests/golden/make_golden_eval.py [--ref /root/reference]
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

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = problems.EVAL_FIXTURES
# the finalised value each objective leaves behind (name of the script's variable)
RESULT_VAR = {"NMSE": "nmse", "L1L1": "l1l1_values", "Normalized-L1L1": "normalized_l1l1_values",
              "GT": "gt_values", "Normalized-GT": "normalized_gt_values", "S-L2": "sl2_values",
              "LASSO": "lasso_values", "LASSO-ALL": "lasso_values"}


def _is_objective_if(node):
    """`if objective == 'NMSE': ...` at the top level of a script."""
    if not isinstance(node, ast.If):
        return False
    t = node.test
    return (isinstance(t, ast.Compare) and isinstance(t.left, ast.Name) and
            t.left.id == "objective" and isinstance(t.comparators[0], ast.Constant) and
            t.comparators[0].value == "NMSE")


def script_nodes(path):
    """(set-up If, per-layer For jj, finalisation If, class DLADMMNet) of a test script."""
    tree = ast.parse(open(path).read())
    batch_for = next(n for n in tree.body if isinstance(n, ast.For) and
                     isinstance(n.target, ast.Name) and n.target.id == "j")
    jj_for = next(n for n in batch_for.body if isinstance(n, ast.For) and
                  isinstance(n.target, ast.Name) and n.target.id == "jj")
    setup = next(n for n in tree.body if _is_objective_if(n) and n.lineno < batch_for.lineno)
    final = next(n for n in tree.body if _is_objective_if(n) and n.lineno > batch_for.lineno)
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "DLADMMNet")
    return setup, jj_for, final, cls


def _code(node, path):
    return compile(ast.Module([node], []), path, "exec")


def make_one(name, c, ref_root):
    torch.Tensor.cuda = lambda self, *a, **k: self
    nn.Module.cuda = lambda self, *a, **k: self
    path = os.path.join(ref_root, c["script"])
    setup, jj_for, final, cls_node = script_nodes(path)
    inp, sd = problems.eval_problem(c)
    m, n, bs, nb, layers = c["m"], c["n"], c["batch_size"], c["n_batches"], c["layers"]
    K = layers
    n_test = bs * nb
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731

    # the test script's model class with the module globals it reads (make_golden_lskm.py)
    ns = dict(torch=torch, nn=nn, F=F, np=np, sqrt=math.sqrt)
    ns.update(alpha=c["alpha"], delta=-99.0, mu_k_method="None", mu_k_param=0.0, layers=layers,
              K=K, args=types.SimpleNamespace(continued=False))
    exec(_code(cls_node, path), ns)
    model = ns["DLADMMNet"](m=m, n=0, d=n, batch_size=bs, A=t(inp["A"]), Z0=t(inp["Z0"]),
                            E0=t(inp["E0"]), L0=t(inp["L0"]), layers=layers)
    model.load_state_dict({k: t(v) for k, v in sd.items()}, strict=True)
    model.eval()

    # reference forward per batch (+ ground truth), exactly as the batch loop calls it (:469-481)
    X_ts, Z_ts, E_ts = inp["X"], inp["Zstar"], inp["Estar"]
    batches = []
    for j in range(nb):
        xb = t(X_ts[:, j * bs:(j + 1) * bs])
        with torch.no_grad():
            Z, E, L, T = model(xb, True, False, False)
            gt = model(xb, False, False, False, K=c["gt_K"]) if c["gt_K"] else None
        batches.append((xb, Z, E, L, T, gt))

    rec = {}
    for obj in c["objectives"]:
        g = dict(torch=torch, np=np, objective=obj, K=K, layers=layers, alpha=c["alpha"],
                 A_tensor=t(inp["A"]), model=model, use_learned=True, use_safeguard=False,
                 n_test=n_test, batch_size=bs, Z_ts=Z_ts, E_ts=E_ts,
                 my_str=lambda o: "{:f}".format(o), print=lambda *a, **k: None)
        exec(_code(setup, path), g)
        for j, (xb, Z, E, L, T, gt) in enumerate(batches):
            g.update(j=j, input_bs_var=xb, Z=Z, E=E, L=L, T=T,
                     Z_label_bs=t(Z_ts[:, j * bs:(j + 1) * bs]),
                     E_label_bs=t(E_ts[:, j * bs:(j + 1) * bs]))
            if gt is not None:
                g.update(Zp=gt[0], Ep=gt[1], Lp=gt[2], Tp=gt[3])
            exec(_code(jj_for, path), g)
        if obj != "LASSO-ALL":   # its finalisation only np.save()s the array to the cwd
            exec(_code(final, path), g)
        rec["obj_" + obj] = np.asarray(g[RESULT_VAR[obj]].detach().numpy(), np.float64)

    # the forward outputs / ground truth the objectives were computed from
    for i, nm in enumerate("ZELT"):
        rec["ref_" + nm] = np.stack([np.stack([s.numpy() for s in b[1 + i]]) for b in batches])
    if c["gt_K"]:
        for i, nm in enumerate("ZELT"):
            rec["gt_" + nm] = np.stack([b[5][i][-1].numpy() for b in batches])
    shas = {k: problems.sha256(v) for k, v in inp.items()}
    shas.update({"sd:" + k: problems.sha256(v) for k, v in sd.items()})
    rec["meta"] = np.array(json.dumps(dict(name=name, case=c, sha256=shas,
                                           torch=torch.__version__, source=c["script"],
                                           lines=dict(setup=setup.lineno, jj=jj_for.lineno,
                                                      final=final.lineno))))
    out = os.path.join(HERE, name + ".npz")
    np.savez_compressed(out, **rec)
    print(f"{name}: {os.path.getsize(out)/1e3:.0f} kB  " +
          "  ".join(f"{o}={np.ravel(rec['obj_' + o])[-1]:.5g}" for o in c["objectives"]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    torch.set_num_threads(8)
    for nm in a.names or list(CASES):
        make_one(nm, CASES[nm], a.ref)


if __name__ == "__main__":
    main()
