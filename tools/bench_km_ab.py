"""A/B timing of forward-path builds on the KM ground truth (test_syn_l1l1_scalar.py:478:
K = 2000 KM iterations, m = 250, d = 500) in ONE process, interleaved per repetition, HIP events
around each call.  --libs: comma list of `main` (the in-tree library) and paths of ablation
builds (tools/ablate_units.py); --batches: the batch sizes; --no-rowsplit adds each library's
path-1 run (plan flag no_rowsplit) as `<lib>:fused`.

    python tools/bench_km_ab.py --libs main,d-ladmm_amd/lib/abl/x/libdladmm_hip.so \
        --batches 20,4096,8192 [--reps 3] [--K 2000]
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
    ap.add_argument("--batches", default="20,1000,4096")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--K", type=int, default=2000)
    ap.add_argument("--no-rowsplit", action="store_true")
    a = ap.parse_args()
    dl = importlib.import_module("d-ladmm_amd")
    ops = importlib.import_module("d-ladmm_amd.ops")
    L = importlib.import_module("d-ladmm_amd._lib")
    dev = torch.device("cuda", 0)
    M, N = 250, 500
    Bs = [int(b) for b in a.batches.split(",")]
    A, X, Z0, E0, L0 = bench.synth(M, N, max(Bs), 0, dev)
    libs = {}
    for spec in a.libs.split(","):
        L._LIB = None
        L.LIB_PATH = os.path.join(ROOT, "d-ladmm_amd", "lib", "libdladmm_hip.so") \
            if spec == "main" else os.path.join(ROOT, spec)
        libs[spec] = L.lib()
    modes = [(s, False) for s in libs] + ([(s, True) for s in libs] if a.no_rowsplit else [])
    nets = {}
    for B in Bs:
        nets[B] = dl.DLADMMNetLSKM(m=M, n=0, d=N, batch_size=B, A=A,
                                   Z0=Z0[:, :B].contiguous(), E0=E0[:, :B].contiguous(),
                                   L0=L0[:, :B].contiguous(), layers=20, alpha=0.01).cuda()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {(s, f, B): [] for s, f in modes for B in Bs}
    for rep in range(a.reps + 1):
        for B in Bs:
            xb = X[:, :B].contiguous()
            for s, f in modes:
                L._LIB = libs[s]
                torch.cuda.synchronize()
                ev0.record()
                with ops.plan_flags(no_rowsplit=f):
                    out = nets[B](xb, False, False, False, K=a.K)
                ev1.record()
                torch.cuda.synchronize()
                if rep:
                    times[(s, f, B)].append(ev0.elapsed_time(ev1))
                del out
    res = {}
    for (s, f, B), t in times.items():
        res.setdefault(s + (":fused" if f else ""), {})[str(B)] = {
            "median_ms": float(np.median(t)), "us_per_step": float(np.median(t)) * 1e3 / a.K}
    res["config"] = dict(m=M, n=N, K=a.K, reps=a.reps)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
