"""Training-step benchmark: one reference training step
(main_syn_l1l1_scalar.py:269-299 -- zero_grad, forward, per-layer L1L1 loss with decay, backward,
Adam step) of the V4 model on one MI355X, with the forward and backward of the drop-in module
timed separately by HIP events on the current stream.

    python tools/bench_train.py [--batch B] [--steps K] [--warmup W] [--m 256 --n 512 --layers 15]

Prints one JSON line.  FLOP model per sample: forward (4K+2)mn; backward 6mn per layer -- what the
V4 backward performs with the forward's saved A Z_k and Z_k mask (BK2 A^T gP, BK3 M^T gU, weight
gradient gU Var^T): `backward_frac_fp32_mfma` is that performed fraction of the fp32 MFMA peak.
`*_reference_equiv` counts the 10mn per layer a recomputing backward forms (BK1 A Z_k, BK2's
M Var), for comparison only.  The loss's own torch.mm(A, Z_k) and its backward (4mn per layer,
hipBLASLt) are counted separately.
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
import bench  # noqa: E402  (synthetic inputs)

PEAK = 157.3e12


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--layers", type=int, default=15)
    ap.add_argument("--alpha", type=float, default=0.001)
    ap.add_argument("--variant", default="v4", choices=["v1", "v2", "v3", "v4", "v5", "v6"],
                    help="model variant (v6: LASSO objective); the torch-op loss is V4's L1L1")
    ap.add_argument("--lena-loss", action="store_true",
                    help="V1 with main_lena.py:221-228's loss (torch ops over the returned Z_k, "
                         "E_k and L_k: cotangents of Z, E and L reach the backward), alpha 0.45")
    ap.add_argument("--precision", default="f32", choices=["f32", "f32_split"],
                    help="forward GEMM precision (f32_split: the split-f16 fused forward, which "
                         "saves its A Z_k for the fp32 backward)")
    ap.add_argument("--adam-fused", action="store_true",
                    help="torch.optim.Adam(fused=True) instead of the reference's default Adam")
    ap.add_argument("--lena-fused", action="store_true",
                    help="main_lena.py:221-228's loss as net.training_loss(kind='lena') (fused: "
                         "dladmm_lena_f32 + the reverse sweep with E / L cotangents), alpha 0.45")
    ap.add_argument("--graph", action="store_true",
                    help="also time the whole step (zero_grad, forward, loss, backward, Adam with "
                         "capturable=True) captured once as a HIP graph and replayed (torch's "
                         "whole-network recipe): the step without the Python / launch overhead")
    ap.add_argument("--fused-loss", action="store_true",
                    help="net.training_loss (objective fused into the kernels) instead of the "
                         "reference's torch-op loss over the returned Z_k")
    return ap


def run(a) -> dict:
    """One training-step measurement (the parsed options of parser()); returns the JSON dict."""
    dl = importlib.import_module("d-ladmm_amd")
    dev = torch.device("cuda", 0)
    m, n, K, B = a.m, a.n, a.layers, a.batch
    A, X, Z0, E0, L0 = bench.synth(m, n, B, 0, dev)
    net = dl.VARIANTS[a.variant](m=m, n=0, d=n, batch_size=B, A=A, Z0=Z0, E0=E0, L0=L0,
                                 layers=K)
    net.precision = a.precision
    kind = "lasso" if a.variant == "v6" else "l1l1"
    if a.lena_fused:
        a.alpha = 0.45
    if a.lena_loss and a.variant != "v1":
        raise SystemExit("--lena-loss is main_lena.py's (V1)")
    if not a.fused_loss and not a.lena_loss and not a.lena_fused and a.variant != "v4":
        raise SystemExit("the torch-op loss leg is V4's (main_syn_l1l1_scalar.py)")
    At = A.t()

    def dual_gap(x, al):  # main_lena.py:145-147
        return torch.nn.functional.softplus(x - al) + torch.nn.functional.softplus(-x - al)
    opt = torch.optim.Adam(net.parameters(), lr=0.005,
                           **({"fused": True} if a.adam_fused else {}),
                           **({"capturable": True} if a.graph else {}))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]

    def step(timed):
        opt.zero_grad(set_to_none=not a.graph)
        if timed:
            ev[0].record()
        coeffs = [0.6 if k < K - 1 else 1.0 for k in range(K)]
        if a.lena_fused:
            tot, _ = net.training_loss(X, a.alpha, [1.0] * K, "lena")
            if timed:
                ev[1].record()
                ev[2].record()
        elif a.fused_loss:
            tot, _ = net.training_loss(X, a.alpha, coeffs, kind)
            if timed:
                ev[1].record()
                ev[2].record()
        elif a.lena_loss:
            Z, E, L = net(X)
            if timed:
                ev[1].record()
            tot = 0
            for k in range(K):  # main_lena.py:221-228
                tot = tot + (0.45 * torch.mean(torch.abs(Z[k])) + torch.mean(torch.abs(E[k])) +
                             torch.mean(dual_gap(torch.mm(At, L[k]), 0.45)) +
                             torch.mean(dual_gap(L[k], 1)) + torch.mean(L[k] * X))
            if timed:
                ev[2].record()
        else:
            Z, E, L, T = net(X)
            if timed:
                ev[1].record()
            tot = 0
            for k in range(K):  # main_syn_l1l1_scalar.py:283-296
                lk = a.alpha * torch.sum(torch.abs(Z[k]), dim=0).mean() + \
                    torch.sum(torch.abs(X - torch.mm(A, Z[k])), dim=0).mean()
                tot = tot + lk * coeffs[k]
            if timed:
                ev[2].record()
        tot.backward()
        if timed:
            ev[3].record()
        opt.step()
        return tot

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize()
    fw, lo, bw, tot_t = [], [], [], []
    for _ in range(a.steps):
        t0 = time.perf_counter()
        loss = step(True)
        torch.cuda.synchronize()
        tot_t.append(time.perf_counter() - t0)
        fw.append(ev[0].elapsed_time(ev[1]))
        lo.append(ev[1].elapsed_time(ev[2]))
        bw.append(ev[2].elapsed_time(ev[3]))
    med = lambda v: float(np.median(v))  # noqa: E731
    flop_f = (4 * K + 2) * m * n * B
    flop_b = 6 * K * m * n * B       # performed
    flop_r = 10 * K * m * n * B      # reference-equivalent (recomputing backward)
    res = {
        "metric": f"training steps/s ({a.variant.upper()} forward + "
                  f"{'main_lena' if a.lena_loss or a.lena_fused else kind} loss + backward + Adam)",
        "variant": a.variant, "precision": a.precision, "adam_fused": a.adam_fused,
        "loss_path": ("main_lena.py:221-228 fused (net.training_loss kind='lena')"
                      if a.lena_fused else "fused (net.training_loss)" if a.fused_loss else
                      "main_lena.py:221-228 torch ops on Z_k, E_k, L_k" if a.lena_loss else
                      "torch ops on Z_k"),
        "batch": B, "m": m, "n": n, "layers": K,
        "step_ms": med(tot_t) * 1e3,
        "samples_per_s": B / med(tot_t),
        "forward_ms": med(fw), "loss_ms": med(lo), "backward_ms": med(bw),
        "forward_tflops": flop_f / (med(fw) * 1e-3) / 1e12,
        # performed: 6 mn per layer (saved A Z_k and Z_k mask) -- the headline
        "backward_tflops": flop_b / (med(bw) * 1e-3) / 1e12,
        "backward_frac_fp32_mfma": flop_b / (med(bw) * 1e-3) / PEAK,
        # note only: the 10 mn per layer a recomputing backward would form
        "backward_tflops_reference_equiv": flop_r / (med(bw) * 1e-3) / 1e12,
        "backward_frac_fp32_mfma_reference_equiv": flop_r / (med(bw) * 1e-3) / PEAK,
        "loss": float(loss.detach()),
    }
    if a.graph:
        # torch's whole-network recipe: warm up on a side stream, capture one step (zero_grad
        # keeps the .grad buffers the graph writes), replay.  The eager loop's last loss keeps its
        # autograd graph (and AccumulateGrad nodes bound to the default stream) alive: drop it
        del loss
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                step(False)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            gl = step(False)
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        res.update({"graph_step_ms": dt * 1e3, "graph_samples_per_s": B / dt,
                    "graph_loss": float(gl.detach()),
                    "graph_note": "the whole step replayed from one HIP graph (Adam "
                                  "capturable=True; eager numbers above use the same optimizer)"})
    del opt, net
    return res


def main():
    print(json.dumps(run(parser().parse_args())), flush=True)


if __name__ == "__main__":
    main()
