"""Rows f2 / f3 at the reference test script's own workload (test_syn_l1l1_scalar.py:24-54,
385-387, 466-531): m = 250, d = 500, n_test = 1,000 test samples in batches of 20, a 20-layer
learned model, and the K = 2000 KM run that gives the Normalized / GT objectives their ground
truth (:478).  One MI355X, HIP events around each call, inputs resident, median of --reps.

  km_gt_b20      model(x, False, False, False, K=2000) on one 20-column batch, as the script
                 calls it (50 of them per test pass)
  km_gt_b1000    the same on the whole test set as one 1,000-column batch (columns are
                 independent: the same values)
  lskm_sg_b1000  model(x, True, True, False): 20 learned layers, safeguarded (EMA mu), counts
  eval_b1000     Evaluator("Normalized-L1L1").add_batch over the 20 layers (with ground truth)

FLOP per KM call = (4K + 2) m n B (two GEMMs per step + T_0); fp32 MFMA peak 157.3 TF/s.
cpu: oracle/dladmm_oracle_lskm.py (the reference's op sequence in numpy, BLAS threads as the
box grants) on a bounded sample -- K = 200 at B = 20, scaled to K = 2000 per call.

    python tools/bench_eval.py [--reps 5] [--no-cpu]   -> one JSON line
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (synthetic inputs, gen_syn_data distribution)

M, N, LAYERS, KGT, ALPHA = 250, 500, 20, 2000, 0.01
PEAK = 157.3e12


def timed(fn, reps):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        ev0.record()
        out = fn()
        ev1.record()
        torch.cuda.synchronize()
        ts.append(ev0.elapsed_time(ev1))
        del out
    return float(np.median(ts)), [round(t, 4) for t in ts]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--ab", action="store_true",
                    help="also the KM lines on path 1 (plan flag no_rowsplit) and at B = 4,096")
    ap.add_argument("--per-layer", action="store_true",
                    help="also the KM lines on the per-layer kernels (plan flag per_layer)")
    a = ap.parse_args()
    dl = importlib.import_module("d-ladmm_amd")
    obj = importlib.import_module("d-ladmm_amd.objectives")
    dev = torch.device("cuda", 0)
    res = {}
    torch.manual_seed(1126)
    A, X4, Z04, E04, L04 = bench.synth(M, N, 4096, 0, dev)   # the KM lines take B columns
    X, Z0, E0, L0 = (t[:, :1000].contiguous() for t in (X4, Z04, E04, L04))
    net = dl.DLADMMNetLSKM(m=M, n=0, d=N, batch_size=1000, A=A, Z0=Z0, E0=E0, L0=L0,
                           layers=LAYERS, alpha=ALPHA, mu_k_method="EMA", mu_k_param=0.5)
    net.cuda()

    ops = importlib.import_module("d-ladmm_amd.ops")

    def km_line(B, per_layer=False, no_rowsplit=False):
        nb = dl.DLADMMNetLSKM(m=M, n=0, d=N, batch_size=B, A=A, Z0=Z04[:, :B].contiguous(),
                              E0=E04[:, :B].contiguous(), L0=L04[:, :B].contiguous(),
                              layers=LAYERS, alpha=ALPHA)
        nb.cuda()
        xb = X4[:, :B].contiguous()
        def call():
            with ops.plan_flags(per_layer=per_layer, no_rowsplit=no_rowsplit):
                return nb(xb, False, False, False, K=KGT)
        ms, runs = timed(call, a.reps)
        flop = (4 * KGT + 2) * M * N * B
        return {"ms_per_call": ms, "runs_ms": runs, "samples_per_s": B / ms * 1e3,
                "tflops": flop / ms / 1e9, "frac_fp32_mfma": flop / ms / 1e-3 / PEAK,
                "us_per_km_step": ms * 1e3 / KGT}

    res["km_gt_b20"] = km_line(20)
    res["km_gt_b20"]["test_pass_s"] = res["km_gt_b20"]["ms_per_call"] * 50 / 1e3
    res["km_gt_b1000"] = km_line(1000)
    if a.ab:   # the same calls on path 1 (the fused kernel's 64-column workgroups)
        res["km_gt_b20_fused"] = km_line(20, no_rowsplit=True)
        res["km_gt_b1000_fused"] = km_line(1000, no_rowsplit=True)
        res["km_gt_b4096"] = km_line(4096)
        res["km_gt_b4096_fused"] = km_line(4096, no_rowsplit=True)
    if a.per_layer:
        res["km_gt_b20_per_layer"] = km_line(20, True)
        res["km_gt_b1000_per_layer"] = km_line(1000, True)
    ms, runs = timed(lambda: net(X, True, True, False), a.reps)
    res["lskm_sg_b1000"] = {"ms_per_call": ms, "runs_ms": runs, "samples_per_s": 1000 / ms * 1e3,
                            "layers": LAYERS, "mu": "EMA 0.5"}
    Z, E, L, T = net(X, True, False, False)
    Zp, Ep, Lp, Tp = net(X, False, False, False, K=KGT)
    gt = (Zp[-1], Ep[-1], Tp[-1])

    def ev():
        e = obj.Evaluator("Normalized-L1L1", LAYERS, ALPHA, n_test=1000)
        e.add_batch(X, Z, E, T=T, gt=gt)
        return e.acc
    ms, runs = timed(ev, a.reps)
    res["eval_b1000"] = {"ms_per_call": ms, "runs_ms": runs, "objective": "Normalized-L1L1",
                         "layers": LAYERS}
    if not a.no_cpu:
        from oracle import dladmm_oracle_lskm as ol
        Kc, Bc = 200, 20
        Xc = X[:, :Bc].cpu().numpy()
        args = (Xc, A.cpu().numpy(), Z0[:, :Bc].cpu().numpy(), E0[:, :Bc].cpu().numpy(),
                L0[:, :Bc].cpu().numpy(), {}, LAYERS, False, False, False, Kc, ALPHA)
        ol.lskm_forward(*args)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            ol.lskm_forward(*args)
            ts.append(time.perf_counter() - t0)
        per_call = float(np.median(ts)) * KGT / Kc
        res["cpu_baseline"] = {"kind": "port", "sample": f"oracle/dladmm_oracle_lskm.py KM, "
                               f"K={Kc} at B={Bc}, median of 3, scaled to K={KGT}",
                               "ms_per_call_b20": per_call * 1e3,
                               "samples_per_s": Bc / per_call,
                               "threads": torch.get_num_threads()}
    res["config"] = dict(m=M, n=N, layers=LAYERS, K_gt=KGT, alpha=ALPHA, reps=a.reps,
                         device=torch.cuda.get_device_name(0))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
