"""Generate tests/golden/bf16_*.npz: the REFERENCE forward with bf16-operand GEMMs (BASELINE config 5,
"bf16 forward + fp32 dual accumulator, tolerance re-stated").

Build container only (reads /root/reference).  The reference has no bf16 mode; config 5 asks for
the reference algorithm with bf16 matrix operands and fp32 state.  This script runs the reference
classes themselves (ast-extracted exactly as make_golden.py does) with their two GEMM entry points
redefined to that arithmetic:

  * `Tensor.mm`  (self.A.mm(Z), main_lena.py:70,73-74,87-88; main_syn_l1l1_scalar.py:92,96,99)
  * `F.linear`   (what nn.Linear fc[k](Var.t()) calls, main_lena.py:72,86)

each rounding both operands to bf16 (round to nearest even, torch's own fp32 -> bf16 conversion),
accumulating the exact products in fp64 and returning fp32.  Every other operation (the shrinks,
AXPYs, the E/L/T updates, the evaluation order) is the reference's own fp32 code.  The same
classes are also run unmodified in fp32, so each fixture carries s_k = the distance bf16 operand
rounding puts between the two, and once more with the bf16 products accumulated in fp32, giving
d_k = the distance accumulation order alone puts between two valid bf16 implementations (it grows
with depth where the iteration amplifies rounding, as at the config-5 shape) -- the yardsticks
the re-stated tolerance is written in (tests/test_gpu_bf16.py).

Usage:  python tests/golden/make_golden_bf16.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import problems  # noqa: E402
from make_golden import load_ref_cls, nrel, run_ref  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def _b(x):
    return x.to(torch.bfloat16).to(torch.float64)


def bf16_gemms(acc=torch.float64):
    """Patch the reference's GEMM entry points to bf16 operands, accumulated in `acc` (fp64: the
    exact products' sum; fp32: a second valid implementation whose distance from the first, d_k,
    measures what accumulation order alone does to this arithmetic); returns an undo function."""
    mm0, lin0 = torch.Tensor.mm, F.linear

    def mm(a, b):
        return mm0(_b(a).to(acc), _b(b).to(acc)).to(torch.float32)

    def linear(inp, weight, bias=None):
        assert bias is None
        return mm0(_b(inp).to(acc), _b(weight).to(acc).t()).to(torch.float32)

    torch.Tensor.mm = mm
    F.linear = linear

    def undo():
        torch.Tensor.mm = mm0
        F.linear = lin0
    return undo


def make_one(name, defn, ref_root):
    torch.Tensor.cuda = lambda self, *a, **k: self
    nn.Module.cuda = lambda self, *a, **k: self
    variant = defn["variant"]
    cls = load_ref_cls(os.path.join(ref_root, problems.VARIANT_SOURCES[variant]))
    inp, sd = problems.build_problem(defn)
    K = defn["K"]
    out32, keys = run_ref(cls, inp, sd, K, torch.float32)
    undo = bf16_gemms()
    try:
        outb, _ = run_ref(cls, inp, sd, K, torch.float32)
    finally:
        undo()
    undo = bf16_gemms(torch.float32)
    try:
        outa, _ = run_ref(cls, inp, sd, K, torch.float32)
    finally:
        undo()
    rec = {}
    names = ["Z", "E", "L", "T"][: len(out32)]
    for nm, sb, s32, sa in zip(names, outb, out32, outa):
        rec[nm] = np.stack([t.numpy() for t in sb]).astype(np.float32)
        rec["f32_" + nm] = np.stack([t.numpy() for t in s32]).astype(np.float32)
        rec["s_" + nm] = np.array([nrel(rec[nm][k], rec["f32_" + nm][k])
                                   for k in range(rec[nm].shape[0])])
        rec["d_" + nm] = np.array([nrel(sa[k].numpy(), rec[nm][k])
                                   for k in range(rec[nm].shape[0])])
    shas = {k: problems.sha256(v) for k, v in inp.items()}
    shas.update({"sd:" + k: problems.sha256(v) for k, v in sd.items()})
    rec["meta"] = np.array(json.dumps(dict(name=name, defn=defn, keys=keys, sha256=shas,
                                           torch=torch.__version__,
                                           source=problems.VARIANT_SOURCES[variant])))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **rec)
    print(f"{name:18s} {os.path.getsize(path)/1e3:8.1f} kB  max s_k " +
          " ".join(f"{nm}={float(np.max(rec['s_' + nm])):.2e}" for nm in names) + "  max d_k " +
          " ".join(f"{nm}={float(np.max(rec['d_' + nm])):.2e}" for nm in names))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    torch.set_num_threads(8)
    for nm in a.names or list(problems.BF16_FIXTURES):
        make_one(nm, problems.BF16_FIXTURES[nm], a.ref)


if __name__ == "__main__":
    main()
