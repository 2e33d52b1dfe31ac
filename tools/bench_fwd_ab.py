"""A/B timing of forward builds in ONE process (interleaved per repetition, HIP events around
each dladmm_forward call): V4 (or --variant) at m x n, K layers, the fused L1L1 objective
(--no-loss: none), every layer written, for each batch in --batches, each library in --libs
(`main` = the in-tree library, or ablation builds from tools/ablate_units.py), on the default plan
and (--no-rowsplit) with the plan flag no_rowsplit.  Prints one JSON line (median ms, path).

    python tools/bench_fwd_ab.py --libs main,d-ladmm_amd/lib/abl/x/libdladmm_hip.so \
        --batches 10000,16384 [--reps 10] [--no-rowsplit | --flag-set 0,128,64]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="main")
    ap.add_argument("--batches", default="10000")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variant", default="v4")
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--layers", type=int, default=15)
    ap.add_argument("--no-loss", action="store_true")
    ap.add_argument("--no-rowsplit", action="store_true")
    ap.add_argument("--flag-set", default="",
                    help="comma-separated plan-flag values to compare, e.g. 0,128,64 "
                         "(default plan, no_xsplit, no_rowsplit); overrides --no-rowsplit")
    a = ap.parse_args()
    dl = importlib.import_module("d-ladmm_amd")
    ops = importlib.import_module("d-ladmm_amd.ops")
    L = importlib.import_module("d-ladmm_amd._lib")
    dev = torch.device("cuda", 0)
    Bs = [int(b) for b in a.batches.split(",")]
    libs = {}
    for spec in a.libs.split(","):
        L._LIB = None
        L.LIB_PATH = os.path.join(ROOT, "d-ladmm_amd", "lib", "libdladmm_hip.so") \
            if spec == "main" else os.path.join(ROOT, spec)
        libs[spec] = L.lib()
    if a.flag_set:
        modes = [(s, int(f)) for s in libs for f in a.flag_set.split(",")]
    else:
        modes = [(s, 0) for s in libs] + \
            ([(s, L.F_NO_ROWSPLIT) for s in libs] if a.no_rowsplit else [])
    calls = {}
    torch.manual_seed(1126)
    for B in Bs:
        A, X, Z0, E0, L0 = bench.synth(a.m, a.n, B, 0, dev)
        net = dl.VARIANTS[a.variant](m=a.m, n=0, d=a.n, batch_size=B, A=A, Z0=Z0, E0=E0,
                                     L0=L0, layers=a.layers).cuda().requires_grad_(False)
        calls[B] = (net, X)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {(s, f, B): [] for s, f in modes for B in Bs}
    paths = {}
    for rep in range(a.reps + 1):
        for B in Bs:
            net, X = calls[B]
            tables = net._tables(dev)
            W = [w.detach() for w in net._weights()]
            for s, f in modes:
                L._LIB = libs[s]
                torch.cuda.synchronize()
                ev0.record()
                r = ops.dladmm_forward(net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0,
                                       keep_all=True, want_T=True,
                                       loss_kind=0 if a.no_loss else L.LOSS_L1L1,
                                       flags=f, **tables)
                ev1.record()
                torch.cuda.synchronize()
                paths[(s, f, B)] = r.path
                if rep:
                    times[(s, f, B)].append(ev0.elapsed_time(ev1))
                del r
    res = {}
    for (s, f, B), t in times.items():
        res.setdefault(s + (f":flags={f}" if f else ""), {})[str(B)] = {
            "median_ms": float(np.median(t)), "min_ms": float(np.min(t)), "path": paths[(s, f, B)]}
    res["config"] = dict(variant=a.variant, m=a.m, n=a.n, K=a.layers, reps=a.reps,
                         loss=not a.no_loss)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
