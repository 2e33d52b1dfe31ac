"""Benchmark: samples/s through the K=15 D-LADMM forward (m=256, n=512) on MI355X.

Workload (BASELINE.json configs[1]/north_star): the reference's V4 model
(main_syn_l1l1_scalar.py:34-131) at m=256, n=512, K=15, B=65,536 columns per GPU, synthetic inputs
with the gen_syn_data.py distribution generated on device, reference-init parameters.  One "step"
= one complete forward with every layer's Z, E, L and T written (the reference's return lists),
the per-layer L1L1 objective of the training loop fused in, and (N > 1) one RCCL all-reduce of
the [K, 2] objective sums.  Batch is sharded across ranks (weak scaling: B per GPU fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu-baseline]

Prints ONE JSON line (rank 0).  Roofline of the dominant kernel (the fused K-layer kernel):
algorithmic FLOP per launch (4K+2)*m*n*B over its average duration measured here with
HIP events recorded on the launch stream around the kernel itself; peak = 157.3 TF/s fp32 MFMA.
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
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "samples/sec through d=15 D-LADMM forward (m=256,n=512); %HBM-roofline"
PEAK_F32_MFMA = 157.3e12   # MI355X_MICROARCH.md: fp32 matrix 157.3 TF/s (spec; 155 measured)
PEAK_HBM = 8.0e12          # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
PEAK_BF16_MFMA = 2.5e15    # MI355X_MICROARCH.md: ~2.5 PF/s dense bf16 MFMA


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536, help="columns per GPU")
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--layers", type=int, default=15)
    ap.add_argument("--variant", default="v4", choices=["v4", "v6"],
                    help="v4 = main_syn_l1l1_scalar.py (configs 1-3); v6 = main_syn_lasso_scalar.py "
                         "(config 4: --m 512 --n 2048 --layers 40)")
    ap.add_argument("--alpha", type=float, default=0.001)
    ap.add_argument("--lean", action="store_true", help="write only the last layer (not default)")
    ap.add_argument("--precision", default="f32", choices=["f32", "f32_split", "bf16"],
                    help="f32_split = fp32 GEMMs on the f16 matrix cores (exact hi/lo split, 3 "
                         "products, fp32 accumulation); bf16 = BASELINE config 5 mode (bf16 MFMA "
                         "operands, fp32 state): --precision bf16 --m 1024 --n 4096 --batch 16384")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-split", action="store_true",
                    help="skip the secondary f32_split measurement of the f32 headline run")
    ap.add_argument("--cpu-batch", type=int, default=8192, help="columns of the CPU sample")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    return ap.parse_args()


def synth(m, n, B, seed, dev):
    """gen_syn_data.py:14-47 distribution on device: A column-normalised N(0,1) (same on every
    rank), Z*, E* Bernoulli(0.1)*N(0,1), X = A Z* + E*; Z0 = U(0,1)/n, E0 = L0 = 0."""
    g = torch.Generator(device=dev)
    g.manual_seed(1126)
    A = torch.randn(m, n, generator=g, device=dev)
    A = A / A.pow(2).sum(0, keepdim=True).sqrt()
    g.manual_seed(1126 + 7919 * (seed + 1))
    zs = (torch.rand(n, B, generator=g, device=dev) < 0.1) * torch.randn(n, B, generator=g,
                                                                        device=dev)
    es = (torch.rand(m, B, generator=g, device=dev) < 0.1) * torch.randn(m, B, generator=g,
                                                                        device=dev)
    X = (A @ zs + es).contiguous()
    Z0 = torch.rand(n, B, generator=g, device=dev) / n
    E0 = torch.zeros(m, B, device=dev)
    L0 = torch.zeros(m, B, device=dev)
    del zs, es
    return A, X, Z0, E0, L0


def cpu_baseline(m, n, K, B, variant="v4"):
    """The oracle (CPU restatement of the reference forward, numpy fp32 + BLAS) on a bounded
    sample of the same workload: B columns, median of 3 forwards after 1 warmup."""
    from oracle import dladmm_oracle as oracle
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import problems
    try:
        from threadpoolctl import threadpool_info
        cores = max((d.get("num_threads", 1) for d in threadpool_info()
                     if d.get("user_api") == "blas"), default=1)
    except Exception:  # pragma: no cover
        cores = os.cpu_count()
    inp = problems.make_inputs(m, n, B, 1126)
    sd = problems.make_state_dict(variant, m, n, B, K, inp["A"], 1126)
    args = (variant, inp["X"], inp["A"], inp["Z0"], inp["E0"], inp["L0"], sd, K)
    oracle.forward(*args)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        oracle.forward(*args)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    return {"value": B / t, "unit": "samples/s", "cores": int(cores), "kind": "port",
            "sample": f"oracle/dladmm_oracle.py {variant.upper()} forward, m={m} n={n} K={K}, B={B} columns, "
                      f"fp32 numpy+BLAS, median of 3 after 1 warmup ({t*1e3:.0f} ms/forward)"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU over RCCL ("nccl" on ROCm).  DLADMM_BENCH_BACKEND=gloo rehearses the N > 1
    # control path with several ranks on fewer GPUs (rank r on GPU r % count); never for numbers
    backend = os.environ.get("DLADMM_BENCH_BACKEND", "nccl")
    gpu = local if backend == "nccl" else local % max(torch.cuda.device_count(), 1)
    if world > 1:
        torch.cuda.set_device(gpu)
        dist.init_process_group(backend)
    dev = torch.device("cuda", gpu if world > 1 else 0)
    torch.cuda.set_device(dev)
    dl = importlib.import_module("d-ladmm_amd")

    m, n, K, B = a.m, a.n, a.layers, a.batch
    A, X, Z0, E0, L0 = synth(m, n, B, rank, dev)
    cls = {"v4": dl.DLADMMNetScalar, "v6": dl.DLADMMNetLasso}[a.variant]
    net = cls(m=m, n=0, d=n, batch_size=B, A=A, Z0=Z0, E0=E0, L0=L0, layers=K)
    net.precision = a.precision
    lk = dl._lib.LOSS_L1L1 if a.variant == "v4" else dl._lib.LOSS_LASSO
    net.requires_grad_(False)
    keep_all = not a.lean
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.steps)]
    for e in ev:
        e.record()  # torch creates the hipEvent lazily; make the handles exist
    torch.cuda.synchronize()

    ddist = importlib.import_module("d-ladmm_amd.dist")

    def step(evpair=None):
        r = net.run(X, keep_all=keep_all, loss_kind=lk, kernel_events=evpair)
        # one RCCL all-reduce of the [K, 2] objective sums over xGMI (no-op at N = 1)
        obj = ddist.global_objectives(r.loss_sums, a.alpha, B * world)
        return r, obj

    def timed(precision):
        """W untimed warmup steps, then exactly K timed steps between barrier + synchronize;
        (max-over-ranks wall seconds, mean kernel seconds, objective)."""
        net.precision = precision
        with torch.no_grad():
            for _ in range(a.warmup):
                r, obj = step()
                del r
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                r, obj = step((ev[2 * i], ev[2 * i + 1]))
                del r
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t1 = time.perf_counter()
        elapsed = t1 - t0
        kern = float(np.mean([ev[2 * i].elapsed_time(ev[2 * i + 1])
                              for i in range(a.steps)])) * 1e-3
        if world > 1:
            tt = torch.tensor([elapsed, kern], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed, kern = float(tt[0]), float(tt[1])
        return elapsed, kern, obj

    elapsed, kern_avg, obj = timed(a.precision)
    # the same workload with the fp32 GEMMs on the f16 matrix cores (split-f16, same fp32
    # tolerance tests; tests/test_gpu_split.py), timed the same way beside the headline
    split = None
    if a.precision == "f32" and m <= 256 and n <= 512 and B % 4 == 0 and \
            os.environ.get("DLADMM_PATH", "")[:1] != "l" and not a.no_split:
        s_el, s_kern, s_obj = timed("f32_split")
        # untimed: per-layer norm-relative distance of the split path's Z/E/L/T from the fp32
        # path's on this whole batch (max over layers and outputs)
        with torch.no_grad():
            net.precision = "f32"
            rf = net.run(X, keep_all=keep_all, loss_kind=lk)
            net.precision = "f32_split"
            rs = net.run(X, keep_all=keep_all, loss_kind=lk)
            dev_max = 0.0
            for name in ("Z", "E", "L", "T"):
                tf, ts = getattr(rf, name), getattr(rs, name)
                if tf is None:
                    continue
                for k in range(tf.shape[0]):
                    nf = torch.linalg.vector_norm(tf[k].double())
                    if nf > 0:
                        d = torch.linalg.vector_norm((ts[k] - tf[k]).double()) / nf
                        dev_max = max(dev_max, float(d))
            del rf, rs
            net.precision = a.precision
        split = (s_el, s_kern, float(s_obj.cpu().numpy()[-1]), dev_max)
    obj = obj.cpu().numpy()

    if rank == 0:
        fused = (m <= 256 and n <= 512 and os.environ.get("DLADMM_PATH", "")[:1] != "l"
                 and a.precision in ("f32", "f32_split"))
        path = ("fused-split-f16" if a.precision == "f32_split" else "fused") if fused \
            else "per-layer"
        # split-f16: 3 f16 MFMA products per fp32 product -> the fp32-GEMM ceiling of the
        # scheme is the dense f16 MFMA peak / 3
        peak = {"bf16": PEAK_BF16_MFMA, "f32": PEAK_F32_MFMA,
                "f32_split": PEAK_BF16_MFMA / 3}[a.precision]
        kname = ({"fused": "dladmm::fused_kernel (one launch)",
                  "fused-split-f16": "dladmm::fused_x3_kernel (one launch)"}.get(path) or
                 f"dladmm::layer_kernel x {2 * K + 1} launches (timed together)")
        total = B * world * a.steps
        value = total / elapsed
        flop = (4 * K + 2) * m * n * B                      # per launch (one rank's shard)
        achieved = flop / kern_avg  # noqa
        # algorithmic HBM bytes per sample (SURVEY 8d, V4 API-parity): inputs X,Z0,E0,L0 +
        # outputs Z,E,L (K layers) + T (K+1); weights (K+1)*m*n*4 per launch
        bytes_io = 4 * ((m + n + 2 * m) + K * (n + 2 * m) + (K + 1) * m) if keep_all else \
            4 * ((m + n + 2 * m) + (n + 3 * m))
        bytes_launch = bytes_io * B + (K + 1) * m * n * 4
        traffic = None
        if os.path.exists(a.traffic_json):
            try:
                tj = json.load(open(a.traffic_json))
                if tj.get("workload") == \
                        f"{a.variant} m={m} n={n} K={K} B={B} keep_all={int(keep_all)}":
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        res = {
            "metric": METRIC,
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"f32": "f32",
                      "f32_split": "f32 (GEMMs: exact hi/lo f16 split, 3 f16 MFMA products, "
                                   "f32 accumulate)",
                      "bf16": "bf16 operands / f32 state"}[a.precision],
            "data": "synthetic (gen_syn_data.py distribution generated on device; reference-init "
                    "V4 parameters, random W = 0.4(A^T + 1e-3 N))",
            "config": {
                "workload": f"{net.name()} ({a.variant.upper()}) forward m={m} n={n} K={K} "
                            f"B={B}/GPU, all layers' Z/E/L/T written"
                            f"{'' if keep_all else ' (lean: last only)'} + fused per-layer "
                            f"{'L1L1' if a.variant == 'v4' else 'LASSO'} objective",
                "variant": a.variant, "m": m, "n": n, "layers": K, "batch_per_gpu": B,
                "path": path,
                "global_batch": B * world, "keep_all": keep_all,
                "parallelism": f"batch-shard dp{world} (one RCCL all-reduce of [K,2] sums)",
            },
            "roofline": {
                "bound": "mfma",
                "achieved": achieved / 1e12,
                "peak": peak / 1e12,
                "unit": "TFLOP/s",
                "frac": achieved / peak,
                "traffic": traffic,
                "kernel": kname,
                "kernel_ms": kern_avg * 1e3,
                "flop_per_launch": flop,
                "algorithmic_bytes_per_launch": bytes_launch,
                "hbm_frac_algorithmic": bytes_launch / kern_avg / PEAK_HBM,
            },
            "objective_last_layer": float(obj[-1]),
        }
        if split is not None:
            s_el, s_kern, s_objl, s_dev = split
            s_peak = PEAK_BF16_MFMA / 3
            res["split_f16"] = {
                "precision": "f32_split",
                "note": "same workload, fp32 GEMMs as hi*hi + hi*lo + lo*hi of exactly split "
                        "power-of-two-scaled f16 halves on v_mfma_f32_16x16x32_f16, fp32 "
                        "accumulate; fp32 elementwise state; parity at the fp32 tolerances",
                "value": total / s_el,
                "unit": "samples/s",
                "ms_per_step": s_el / a.steps * 1e3,
                "kernel": "dladmm::fused_x3_kernel (one launch)",
                "kernel_ms": s_kern * 1e3,
                "roofline_mfma": {"achieved": flop / s_kern / 1e12, "peak": s_peak / 1e12,
                                  "unit": "TFLOP/s", "frac": flop / s_kern / s_peak,
                                  "peak_note": "dense f16 MFMA peak / 3 products"},
                "hbm_frac_algorithmic": bytes_launch / s_kern / PEAK_HBM,
                "objective_last_layer": s_objl,
                "max_rel_dev_vs_f32": s_dev,
                "max_rel_dev_note": "max over layers of ||X_split - X_f32|| / ||X_f32|| for X in "
                                    "Z, E, L, T on this batch (parity tolerance: 1e-5)",
            }
        if world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(m, n, K, a.cpu_batch, a.variant)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
