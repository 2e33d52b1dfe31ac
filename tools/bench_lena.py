"""Time dladmm_lena_f32 alone (mode 0: the loss sums; mode 1: the E / L cotangents; mode 2: both) at the
main_lena training shape: V1 m=256 n=512 K=15 B=65,536, synthetic E_k / L_k.  One JSON line.
DLADMM_LIB selects a library (tools/ablate.py --unit dladmm_lena.hip variants)."""
import argparse
import importlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
ops = importlib.import_module("d-ladmm_amd.ops")
dev = torch.device("cuda", 0)
m, n, K, B = 256, 512, 15, a.batch
g = torch.Generator(device=dev).manual_seed(1)
X = torch.randn(m, B, device=dev, generator=g)
A = torch.randn(m, n, device=dev, generator=g) / 16
E = torch.randn(K, m, B, device=dev, generator=g) * 0.1
L = torch.randn(K, m, B, device=dev, generator=g)
coef = torch.ones(K, device=dev)
res = {"shape": [m, n, K, B]}
flop1 = 2.0 * m * n * B * K
for mode in (0, 1, 2):
    ts = []
    for i in range(a.reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.dladmm_lena(X, A, E, L, 0.45, B, coef=None if mode == 0 else coef, sums=mode != 1)
        e1.record()
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(e0.elapsed_time(e1))
    ts.sort()
    ms = ts[len(ts) // 2]
    f = flop1 * (1 if mode == 0 else 2)
    res[f"mode{mode}_ms"] = ms
    res[f"mode{mode}_frac_fp32_mfma"] = f / (ms * 1e-3) / 157.3e12
print(json.dumps(res))
