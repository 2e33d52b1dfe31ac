"""Forward throughput of every model variant at the BASELINE config-2 shape (m=256, n=512, K=15,
B=65,536 columns, all layers' Z/E/L/T written + the fused per-layer objective), one MI355X.

    python tools/bench_variants.py [--batch B] [--steps S] [--variants v1,v2,...]

Prints one JSON line per variant: samples/s, kernel ms (HIP events around the op on its stream),
the kernel's fraction of the fp32 MFMA peak ((4K+2) m n FLOP per sample) and the execution path.
Parameters are the reference inits perturbed (tests/golden/problems.py); W_k = 0.4 (A^T + 1e-3 N).
V1 carries per-sample betas (m x B per layer and beta: 2 GB at this batch), streamed per layer.
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

PEAK = 157.3e12


def build(dl, variant, m, n, K, B, A, Z0, E0, L0, dev):
    cls = dl.VARIANTS[variant]
    extra = {"interval": 3} if variant == "v7p" else {}
    net = cls(m=m, n=0, d=n, batch_size=B, A=A, Z0=Z0, E0=E0, L0=L0, layers=K, **extra).to(dev)
    g = torch.Generator(device="cpu").manual_seed(1126)
    with torch.no_grad():
        for name, p in net.named_parameters():
            if name.startswith("fc"):
                p.copy_((0.4 * (A.t().cpu() + 1e-3 * torch.randn(p.shape, generator=g))).to(dev))
            else:
                p.mul_(1.0 + 0.05 * torch.randn(p.shape, generator=g).to(dev))
    net.requires_grad_(False)
    return net


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--layers", type=int, default=15)
    ap.add_argument("--variants", default="v1,v2,v3,v4,v5,v6,v7")
    a = ap.parse_args()
    dl = importlib.import_module("d-ladmm_amd")
    dev = torch.device("cuda", 0)
    m, n, K, B = a.m, a.n, a.layers, a.batch
    A, X, Z0, E0, L0 = bench.synth(m, n, B, 0, dev)
    lib = dl._lib
    for v in a.variants.split(","):
        net = build(dl, v, m, n, K, B, A, Z0, E0, L0, dev)
        lk = lib.LOSS_LASSO if v == "v6" else lib.LOSS_L1L1
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.steps)]
        for e in ev:
            e.record()  # torch creates the hipEvent lazily; make the handles exist
        with torch.no_grad():
            for _ in range(a.warmup):  # tables, workspace, clocks (as bench.py)
                r = net.run(X, keep_all=True, loss_kind=lk)
                del r
            torch.cuda.synchronize()
            for i in range(a.steps):
                r = net.run(X, keep_all=True, loss_kind=lk, kernel_events=(ev[2 * i], ev[2 * i + 1]))
                del r
            torch.cuda.synchronize()
        ms = float(np.mean([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(a.steps)]))
        flop = (4 * K + 2) * m * n * B
        print(json.dumps({"variant": v, "class": type(net).__name__, "m": m, "n": n, "layers": K,
                          "batch": B, "kernel_ms": ms, "samples_per_s": B / (ms * 1e-3),
                          "tflops": flop / (ms * 1e-3) / 1e12,
                          "frac_fp32_mfma": flop / (ms * 1e-3) / PEAK}), flush=True)
        del net
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
