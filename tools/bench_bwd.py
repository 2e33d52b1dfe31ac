"""A/B timing of backward builds in ONE process (interleaved calls, so box-to-box and run-to-run
clock noise cancel): V4 m=256 n=512 K=15 at B=65,536, the fused L1L1 objective, one saved
forward, then `--reps` rounds of one dladmm_bwd_f32 call per library, each timed with HIP
events on the current stream.

    python tools/bench_bwd.py --libs main,d-ladmm_amd/lib/abl/x/libdladmm_hip.so [--reps 10]

`main` is the in-tree library; --per-layer (plan flag bwd_per_layer) selects the per-layer
kernels for every library.  Prints one JSON line: median / min ms per library.
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
import bench  # noqa: E402  (synthetic inputs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="main")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--layers", type=int, default=15)
    ap.add_argument("--gz", action="store_true",
                    help="per-layer Z cotangents (a loss built from the returned Z_k with torch "
                         "ops, the reference's training loops) instead of the fused objective")
    ap.add_argument("--no-rowsplit", action="store_true",
                    help="forward with the plan flag no_rowsplit (path 1), so a small batch's "
                         "backward runs the 64-column reverse sweep instead of its row-split form")
    ap.add_argument("--per-layer", action="store_true",
                    help="plan flag bwd_per_layer: the per-layer backward kernels")
    ap.add_argument("--flag-set", default="",
                    help="comma-separated forward plan flags to compare with the in-tree library "
                         "(e.g. 0,128,64: bwd paths 3 / 2 / 1 at small batches); overrides --libs")
    a = ap.parse_args()
    dl = importlib.import_module("d-ladmm_amd")
    ops = importlib.import_module("d-ladmm_amd.ops")
    L = importlib.import_module("d-ladmm_amd._lib")
    dev = torch.device("cuda", 0)
    m, n, K, B = 256, 512, a.layers, a.batch
    torch.manual_seed(1126)
    A, X, Z0, E0, L0 = bench.synth(m, n, B, 0, dev)
    net = dl.DLADMMNetScalar(m=m, n=0, d=n, batch_size=B, A=A, Z0=Z0, E0=E0, L0=L0, layers=K)
    net.cuda()
    with torch.no_grad():
        tables = net._tables(dev)
    W = [w.detach() for w in net._weights()]
    args = (net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0)
    fls = [int(f) for f in a.flag_set.split(",")] if a.flag_set else \
        [L.F_NO_ROWSPLIT if a.no_rowsplit else 0]
    fwd = {}
    with torch.no_grad():
        for fl in fls:
            fwd[fl] = ops.dladmm_forward(*args, keep_all=True, want_T=True, want_P=True,
                                         loss_kind=L.LOSS_L1L1, flags=fl, **tables)
    coef = torch.tensor([[1e-3 / B, 1.0 / B]] * K, device=dev)
    kw = dict(loss_kind=L.LOSS_L1L1, loss_coef=coef, **tables)
    if a.gz:
        g = torch.Generator(device=dev).manual_seed(7)
        kw = dict(gZ=[torch.randn(n, B, generator=g, device=dev) / B for _ in range(K)], **tables)
    libs = {}
    for spec in (["main"] if a.flag_set else a.libs.split(",")):
        L._LIB = None
        L.LIB_PATH = os.path.join(ROOT, "d-ladmm_amd", "lib", "libdladmm_hip.so") \
            if spec == "main" else os.path.join(ROOT, spec)
        libs[spec] = L.lib()
    runs = [(s, fl) for s in libs for fl in fls]
    name = (lambda s, fl: f"fwd_flags={fl}") if a.flag_set else (lambda s, fl: s)
    times = {name(s, fl): [] for s, fl in runs}
    paths = {}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rep in range(a.reps + 1):
        for spec, fl in runs:
            L._LIB = libs[spec]
            torch.cuda.synchronize()
            ev0.record()
            with ops.plan_flags(bwd_per_layer=a.per_layer):
                res = ops.dladmm_backward(*args, fwd[fl], **kw)
            bwd_path = res.path
            paths[name(spec, fl)] = res.path
            ev1.record()
            torch.cuda.synchronize()
            if rep:  # the first round warms every library's kernels and workspace
                times[name(spec, fl)].append(ev0.elapsed_time(ev1))
            del res
    out = {s: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)), "bwd_path": paths[s]}
           for s, t in times.items()}
    out["config"] = dict(m=m, n=n, K=K, B=B, reps=a.reps, rev=not a.per_layer, gz=a.gz,
                         no_rowsplit=a.no_rowsplit, bwd_path=bwd_path)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
