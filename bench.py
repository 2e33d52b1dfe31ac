"""Benchmark: samples/s through the K=15 D-LADMM forward (m=256, n=512) on MI355X.

Workload (BASELINE.json configs[1]/north_star): the reference's V4 model
(main_syn_l1l1_scalar.py:34-131) at m=256, n=512, K=15, B=65,536 columns per GPU, synthetic inputs
with the gen_syn_data.py distribution generated on device, reference-init parameters.  One "step"
= one complete forward with every layer's Z, E, L and T written (the reference's return lists),
the per-layer L1L1 objective of the training loop fused in, and (N > 1) one RCCL all-reduce of
the [K, 2] objective sums.  Batch is sharded across ranks: the headline is weak scaling (B per GPU
fixed); `--global-batch G` makes it strong scaling instead (BASELINE config 3: G = 262,144 columns
split by dist.shard_columns over the ranks).  The default run also times config 3's strong-scaling
workload beside the headline (`cfg3_strong`), so every driver run at N = 1/2/4/8 records both
curves, and at N = 1 configs 2 (B = 10,000), 4 (V6 LASSO 512 x 2048, K = 40) and 5 (bf16,
1024 x 4096): `cfg2`, `cfg4`, `cfg5`.  The model is built after torch.manual_seed(1126), so the objective is
reproducible.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B | --global-batch G]
                    [--no-cpu-baseline] [--no-split] [--no-cfg3]

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
    ap.add_argument("--batch", type=int, default=65536, help="columns per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: this many columns in total, split over the ranks by "
                         "dist.shard_columns (BASELINE config 3: 262144)")
    ap.add_argument("--no-cfg3", action="store_true",
                    help="skip the secondary measurements of config 3 (strong scaling, 262,144 "
                         "global columns) and config 2 (B = 10,000, N = 1)")
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--layers", type=int, default=15)
    ap.add_argument("--variant", default="v4", choices=["v4", "v6", "v1"],
                    help="v4 = main_syn_l1l1_scalar.py (configs 1-3); v6 = main_syn_lasso_scalar.py "
                         "(config 4: --m 512 --n 2048 --layers 40); v1 = main_lena.py's "
                         "DLADMMNet (per-sample betas, forward only)")
    ap.add_argument("--alpha", type=float, default=0.001)
    ap.add_argument("--lean", action="store_true", help="write only the last layer (not default)")
    ap.add_argument("--precision", default="f32", choices=["f32", "f32_split", "bf16"],
                    help="f32_split = fp32 GEMMs on the f16 matrix cores (exact hi/lo split, 3 "
                         "products, fp32 accumulation); bf16 = BASELINE config 5 mode (bf16 MFMA "
                         "operands, fp32 state): --precision bf16 --m 1024 --n 4096 --batch 16384")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-train", action="store_true",
                    help="skip the training-step line (SURVEY row f1: V4 forward + fused L1L1 "
                         "objective + reverse-sweep backward + Adam at the headline shape)")
    ap.add_argument("--no-split", action="store_true",
                    help="skip the secondary f32_split measurement of the f32 headline run")
    ap.add_argument("--cpu-batch", type=str, default="10000,65536",
                    help="comma-separated batches of the CPU baseline (BASELINE.md: 10,000 and "
                         "65,536)")
    ap.add_argument("--cpu-runs", type=int, default=5, help="timed CPU forwards (median)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--launch-selftest", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def synth(m, n, B, seed, dev, cols=None):
    """gen_syn_data.py:14-47 distribution on device: A column-normalised N(0,1) (same on every
    rank), Z*, E* Bernoulli(0.1)*N(0,1), X = A Z* + E*; Z0 = U(0,1)/n, E0 = L0 = 0.
    cols = (c0, c1): keep only that column shard of the B-column batch (strong scaling: every rank
    generates the same global batch and keeps its own columns)."""
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
    del zs, es
    if cols is not None:
        c0, c1 = cols
        X, Z0 = X[:, c0:c1].contiguous(), Z0[:, c0:c1].contiguous()
        B = c1 - c0
    E0 = torch.zeros(m, B, device=dev)
    L0 = torch.zeros(m, B, device=dev)
    return A, X, Z0, E0, L0


def host_info():
    """CPU model, physical cores and the CPUs this process may run on (GPU box: a share)."""
    model, phys = "unknown", set()
    try:
        cur = {}
        for line in open("/proc/cpuinfo"):
            if ":" not in line:
                if cur:
                    phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
                continue
            k, v = (x.strip() for x in line.split(":", 1))
            cur[k] = v
            if k == "model name":
                model = v
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:  # pragma: no cover
        pass
    return dict(cpu_model=model, physical_cores=len(phys), logical_cpus=os.cpu_count(),
                cpus_allowed=len(os.sched_getaffinity(0)))


def granted_cores():
    """The CPU threads this process is granted and how that was decided: the cgroup v2 quota
    (/sys/fs/cgroup/cpu.max "quota period") when one is set, else the scheduler affinity,
    capped by OMP_NUM_THREADS when the environment sets it (the GPU box sets 16: its CPU share
    per GPU)."""
    raw = None
    quota = None
    try:
        raw = open("/sys/fs/cgroup/cpu.max").read().strip()
        q, per = raw.split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if quota is not None:
        cores, rule = min(quota, aff), "cgroup cpu.max quota"
    elif omp and omp.isdigit() and int(omp) > 0:
        cores, rule = min(int(omp), aff), "OMP_NUM_THREADS (no cgroup quota)"
    else:
        cores, rule = aff, "sched affinity (no cgroup quota)"
    return cores, dict(cgroup_cpu_max=raw, affinity_cpus=aff, omp_num_threads=omp, rule=rule)


def cpu_baseline(m, n, K, batches, runs, variant="v4"):
    """The reference's op sequence in torch on the host CPU (oracle/dladmm_torch_cpu.py: the
    reference's ATen ops in its order, duplicate A.mm included, pinned bit for bit to the golden
    fixtures by tests/test_oracle_torch.py), fp32, no_grad, torch.set_num_threads(<granted
    cores>); the same workload (gen_syn_data.py distribution, reference-init parameters) at each
    batch of `batches` (BASELINE.md "CPU baseline": B = 10,000 and 65,536), median of `runs`
    forwards after 1 warmup.  The headline value is the largest batch's."""
    from oracle import dladmm_torch_cpu as tcpu
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import problems
    cores, how = granted_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    per = {}
    try:
        for B in batches:
            A, X, Z0, E0, L0 = synth(m, n, B, 0, torch.device("cpu"))
            sd = problems.make_state_dict(variant, m, n, 1, K, A.numpy(), 1126)
            params = {k: torch.from_numpy(v) for k, v in sd.items()}
            args = (variant, X, A, Z0, E0, L0, params, K)
            tcpu.forward(*args)
            ts = []
            for _ in range(runs):
                t0 = time.perf_counter()
                tcpu.forward(*args)
                ts.append(time.perf_counter() - t0)
            t = float(np.median(ts))
            per[str(B)] = {"value": B / t, "ms_per_forward": t * 1e3,
                           "runs_ms": [x * 1e3 for x in ts]}
            del A, X, Z0, E0, L0, params
    finally:
        torch.set_num_threads(prev)
    h = host_info()
    Bh = str(max(batches))
    return {"value": per[Bh]["value"], "unit": "samples/s", "cores": int(cores), "kind": "port",
            "sample": f"oracle/dladmm_torch_cpu.py {variant.upper()} forward (the reference's "
                      f"ATen op sequence, bit-equal to the reference classes on the golden "
                      f"fixtures), m={m} n={n} K={K}, fp32 no_grad, torch {torch.__version__} "
                      f"with {cores} threads; B = {', '.join(map(str, batches))} columns, median "
                      f"of {runs} after 1 warmup; value = B={Bh}",
            "per_batch": per, "threads": how, "host": h}


def reduce_timing(elapsed, kern, world, dev, use_dist=None):
    """Max over ranks of the wall seconds and of the mean kernel seconds, plus every rank's mean
    kernel seconds in rank order (one MAX all-reduce + one all-gather; nothing at N = 1 unless the
    process group is up anyway)."""
    if not (world > 1 if use_dist is None else use_dist):
        return elapsed, kern, [kern]
    tt = torch.tensor([elapsed, kern], device=dev, dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    allk = [torch.zeros(1, device=dev, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(allk, torch.tensor([kern], device=dev, dtype=torch.float64))
    return float(tt[0]), float(tt[1]), [float(x) for x in allk]


class Workload:
    """One benchmark workload on this rank: the model, its (shard of the) synthetic batch and the
    timed step (forward + the [K, 2] all-reduce)."""

    def __init__(self, dl, a, m, n, K, B_rank, B_global, cols, rank, dev, seed, wscale=None):
        self.dl, self.a = dl, a
        self.B, self.B_global = B_rank, B_global
        gen_B = B_global if cols is not None else B_rank
        A, X, Z0, E0, L0 = synth(m, n, gen_B, seed, dev, cols)
        self.X = X
        cls = {"v4": dl.DLADMMNetScalar, "v6": dl.DLADMMNetLasso, "v1": dl.DLADMMNet}[a.variant]
        torch.manual_seed(1126)   # params seeded -> reproducible objective
        self.net = cls(m=m, n=0, d=n, batch_size=B_rank, A=A, Z0=Z0, E0=E0, L0=L0, layers=K)
        self.net.requires_grad_(False)
        if wscale is not None:   # W = wscale (A^T + 1e-3 N) instead of the reference's 0.4 (...)
            with torch.no_grad():
                for fc in self.net.fc:
                    fc.weight.mul_(wscale / 0.4)
        # V4: the training loop's fused L1L1 objective; V6: LASSO; V1: the bare forward
        # (main_lena.py's objective is a separate pass, dladmm_lena_f32)
        self.lk = {"v4": dl._lib.LOSS_L1L1, "v6": dl._lib.LOSS_LASSO, "v1": 0}[a.variant]
        self.ddist = importlib.import_module("d-ladmm_amd.dist")

    def step(self, keep_all, evpair=None):
        r = self.net.run(self.X, keep_all=keep_all, loss_kind=self.lk, kernel_events=evpair)
        # one RCCL all-reduce of the [K, 2] objective sums over xGMI (no-op at N = 1)
        obj = (self.ddist.global_objectives(r.loss_sums, self.a.alpha, self.B_global)
               if r.loss_sums is not None else torch.zeros(1, dtype=torch.float64))
        self.path = r.path  # the kernel path the library chose (dladmm_fwd_path)
        return r, obj


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU over RCCL ("nccl" on ROCm).  DLADMM_BENCH_BACKEND=gloo rehearses the N > 1
    # control path with several ranks on fewer GPUs (rank r on GPU r % count); never for numbers
    backend = os.environ.get("DLADMM_BENCH_BACKEND", "nccl")
    gpu = local if backend == "nccl" else local % max(torch.cuda.device_count(), 1)
    # DLADMM_BENCH_DIST=1: the process group, barriers and timing collectives at N = 1 too
    # (rehearses the RCCL control path on a one-GPU box)
    use_dist = world > 1 or os.environ.get("DLADMM_BENCH_DIST", "") == "1"
    if use_dist:
        torch.cuda.set_device(gpu)
        dist.init_process_group(backend)
    dev = torch.device("cuda", gpu if world > 1 else 0)
    torch.cuda.set_device(dev)
    dl = importlib.import_module("d-ladmm_amd")
    ddist = importlib.import_module("d-ladmm_amd.dist")

    m, n, K = a.m, a.n, a.layers
    strong = a.global_batch > 0
    keep_all = not a.lean

    def make(strong_b):
        if strong_b:
            c0, c1 = ddist.shard_columns(strong_b, rank, world)
            return Workload(dl, a, m, n, K, c1 - c0, strong_b, (c0, c1), rank, dev, 0)
        return Workload(dl, a, m, n, K, a.batch, a.batch * world, None, rank, dev, rank)

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.steps)]
    for e in ev:
        e.record()  # torch creates the hipEvent lazily; make the handles exist
    torch.cuda.synchronize()

    def timed(w, precision):
        """W untimed warmup steps, then exactly K timed steps between barrier + synchronize;
        (max-over-ranks wall seconds, max-over-ranks mean kernel seconds, every rank's mean
        kernel seconds, objective)."""
        w.net.precision = precision
        with torch.no_grad():
            for _ in range(a.warmup):
                r, obj = w.step(keep_all)
                del r
            torch.cuda.synchronize()
            if use_dist:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                r, obj = w.step(keep_all, (ev[2 * i], ev[2 * i + 1]))
                del r
            torch.cuda.synchronize()
            if use_dist:
                dist.barrier()
            t1 = time.perf_counter()
        elapsed = t1 - t0
        kern = float(np.mean([ev[2 * i].elapsed_time(ev[2 * i + 1])
                              for i in range(a.steps)])) * 1e-3
        elapsed, kern, kerns = reduce_timing(elapsed, kern, world, dev, use_dist)
        return elapsed, kern, kerns, obj

    w = make(a.global_batch if strong else 0)
    B = w.B
    elapsed, kern_avg, kerns, obj = timed(w, a.precision)
    head_path = w.path
    # the same workload with the fp32 GEMMs on the f16 matrix cores (split-f16, same fp32
    # tolerance tests; tests/test_gpu_split.py), timed the same way beside the headline
    split = None
    if a.precision == "f32" and m <= 256 and n <= 512 and B % 4 == 0 and not a.no_split:
        s_el, s_kern, _, s_obj = timed(w, "f32_split")
        assert w.path == 4, f"split leg ran on path {w.path}, not the split-f16 kernel"
        # untimed: per-layer norm-relative distance of the split path's Z/E/L/T from the fp32
        # path's on this whole batch (max over layers and outputs)
        with torch.no_grad():
            net = w.net
            net.precision = "f32"
            rf = net.run(w.X, keep_all=keep_all, loss_kind=w.lk)
            net.precision = "f32_split"
            rs = net.run(w.X, keep_all=keep_all, loss_kind=w.lk)
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
    del w
    # BASELINE config 3 (V4, 262,144 columns in total, batch-sharded) beside the weak headline
    cfg3 = None
    if not strong and not a.no_cfg3 and a.variant == "v4" and a.precision == "f32" and \
            (m, n, K) == (256, 512, 15):
        w3 = make(262144)
        c_el, c_kern, c_kerns, c_obj = timed(w3, "f32")
        cfg3 = dict(value=262144 * a.steps / c_el, ms_per_step=c_el / a.steps * 1e3,
                    kern=c_kern, kerns=c_kerns, B=w3.B, obj=float(c_obj.cpu().numpy()[-1]))
        del w3
    # BASELINE config 2 (V4, B = 10,000 on one GPU) beside the headline at N = 1: on path 5 (the
    # row-split fused kernel, 625 workgroups of 16 columns)
    cfg2 = None
    if world == 1 and not strong and not a.no_cfg3 and a.variant == "v4" and \
            a.precision == "f32" and (m, n, K) == (256, 512, 15) and B != 10000:
        w2 = Workload(dl, a, m, n, K, 10000, 10000, None, rank, dev, rank)
        c_el, c_kern, _, c_obj = timed(w2, "f32")
        cfg2 = dict(value=10000 * a.steps / c_el, ms_per_step=c_el / a.steps * 1e3, kern=c_kern,
                    obj=float(c_obj.cpu().numpy()[-1]), path=w2.path)
        if not a.no_split:   # the same batch on the split-f16 kernel (same fp32 tolerances)
            s_el, s_kern, _, _ = timed(w2, "f32_split")
            cfg2["split"] = (10000 * a.steps / s_el, s_el / a.steps * 1e3, s_kern, w2.path)
        del w2
    # BASELINE configs 4 (V6 LASSO m=512 n=2048 K=40, per-layer kernels) and 5 (bf16 operands,
    # m=1024 n=4096 K=15, 16,384 columns = its 131,072 over 8 GPUs) at N = 1
    cfg45 = {}
    if world == 1 and not strong and not a.no_cfg3 and a.variant == "v4" and \
            a.precision == "f32" and (m, n, K) == (256, 512, 15):
        import copy
        # config 4 at the reference init diverges (V6 at 512 x 2048: the step 0.4 ||A^T A|| ~ 3.6
        # exceeds 2; objective 2.3e27 by layer 40, BENCH_r03): it is timed with the contracting
        # W = 0.1 (A^T + 1e-3 N) instead -- same kernels, same bytes, a finite O(1) objective
        for name, var, prec, (m_, n_, K_, B_), wsc in (
                ("cfg4", "v6", "f32", (512, 2048, 40, 65536), 0.1),
                ("cfg5", "v4", "bf16", (1024, 4096, 15, 16384), None)):
            a_ = copy.copy(a)
            a_.variant = var
            w_ = Workload(dl, a_, m_, n_, K_, B_, B_, None, rank, dev, rank, wscale=wsc)
            c_el, c_kern, _, c_obj = timed(w_, prec)
            cfg45[name] = dict(value=B_ * a.steps / c_el, ms_per_step=c_el / a.steps * 1e3,
                               kern=c_kern, obj=float(c_obj.cpu().numpy()[-1]), path=w_.path,
                               shape=(m_, n_, K_, B_), var=var, prec=prec, wscale=wsc)
            del w_
            torch.cuda.empty_cache()
    # the north_star's primary variant V1 (main_lena.py:16-102, DLADMMNet: per-sample (m, B)
    # betas read by every layer) at the headline shape, forward with every layer's Z/E/L written
    v1 = None
    if world == 1 and not strong and not a.no_cfg3 and a.variant == "v4" and \
            a.precision == "f32" and (m, n, K) == (256, 512, 15):
        import copy
        a1 = copy.copy(a)
        a1.variant = "v1"
        w1 = Workload(dl, a1, m, n, K, B, B, None, rank, dev, rank)
        c_el, c_kern, _, _ = timed(w1, "f32")
        v1 = dict(value=B * a.steps / c_el, ms_per_step=c_el / a.steps * 1e3, kern=c_kern,
                  path=w1.path, B=B)
        if not a.no_split:   # V1 on the split-f16 kernel (round 6; same fp32 tolerances)
            s_el, s_kern, _, _ = timed(w1, "f32_split")
            v1["split"] = (B * a.steps / s_el, s_el / a.steps * 1e3, s_kern, w1.path)
        del w1
        torch.cuda.empty_cache()
    torch.cuda.synchronize()
    # SURVEY row f1 at N = 1: the headline shape's training step (tools/bench_train.py: forward +
    # fused per-layer L1L1 objective + reverse-sweep backward + Adam), timed after everything above
    train = None
    if world == 1 and not strong and not a.no_train and a.variant == "v4" and \
            a.precision == "f32" and (m, n, K) == (256, 512, 15):
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_train
        ta = bench_train.parser().parse_args(["--variant", "v4", "--fused-loss", "--batch", str(B),
                                              "--steps", "10", "--warmup", "3"])
        # a failure here (e.g. out of memory after the legs above) is recorded, never allowed
        # to cost the headline line
        try:
            train = bench_train.run(ta)
        except Exception as e:  # noqa: BLE001
            train = {"error": f"{type(e).__name__}: {e}"}
        torch.cuda.empty_cache()
        if not a.no_split and "error" not in train:
            # the same step on the split-f16 kernels (forward + weight gradient)
            ts = bench_train.parser().parse_args(["--variant", "v4", "--fused-loss", "--batch",
                                                  str(B), "--steps", "10", "--warmup", "3",
                                                  "--precision", "f32_split"])
            try:
                train["split_f16"] = {k: v for k, v in bench_train.run(ts).items()
                                      if k in ("step_ms", "samples_per_s", "forward_ms",
                                               "backward_ms")}
            except Exception as e:  # noqa: BLE001
                train["split_f16"] = {"error": f"{type(e).__name__}: {e}"}
            torch.cuda.empty_cache()
        if "error" not in train:
            # the reference training loop's own batch (main_syn_l1l1_scalar.py -bs 25): the
            # row-split forward and reverse sweep; host-bound at this size
            tr = bench_train.parser().parse_args(["--variant", "v4", "--fused-loss", "--batch",
                                                  "25", "--steps", "50", "--warmup", "5"])
            try:
                train["ref_batch"] = {k: v for k, v in bench_train.run(tr).items()
                                      if k in ("batch", "step_ms", "samples_per_s", "forward_ms",
                                               "backward_ms")}
            except Exception as e:  # noqa: BLE001
                train["ref_batch"] = {"error": f"{type(e).__name__}: {e}"}

    if rank == 0:
        path = {1: "fused", 2: "per-layer", 3: "bf16-tiles", 4: "fused-split-f16"}.get(
            head_path, f"path {head_path}")
        # split-f16: 3 f16 MFMA products per fp32 product -> the fp32-GEMM ceiling of the
        # scheme is the dense f16 MFMA peak / 3
        peak = {"bf16": PEAK_BF16_MFMA, "f32": PEAK_F32_MFMA,
                "f32_split": PEAK_BF16_MFMA / 3}[a.precision]
        kname = ({"fused": "dladmm::fused_kernel (one launch)",
                  "fused-split-f16": "dladmm::fused_x3_kernel (one launch)"}.get(path) or
                 f"dladmm::layer_kernel x {2 * K + 1} launches (timed together)")
        B_global = w_global = (a.global_batch if strong else B * world)
        total = B_global * a.steps
        value = total / elapsed
        flop = (4 * K + 2) * m * n * B                      # per launch (rank 0's shard)
        achieved = flop / kern_avg  # noqa
        bytes_launch = alg_bytes(a.variant, m, n, K, B, keep_all)
        traffic = None
        if os.path.exists(a.traffic_json):
            try:
                tj = json.load(open(a.traffic_json))
                if tj.get("workload") == \
                        f"{a.variant} m={m} n={n} K={K} B={B} keep_all={int(keep_all)}":
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        scal = "strong" if strong else "weak"
        res = {
            "metric": METRIC,
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": scal,
            "vs_baseline": None,
            "dtype": {"f32": "f32",
                      "f32_split": "f32 (GEMMs: exact hi/lo f16 split, 3 f16 MFMA products, "
                                   "f32 accumulate)",
                      "bf16": "bf16 operands / f32 state"}[a.precision],
            "data": "synthetic (gen_syn_data.py distribution generated on device; reference-init "
                    f"{a.variant.upper()} parameters after torch.manual_seed(1126), "
                    "W = 0.4(A^T + 1e-3 N))",
            "config": {
                "workload": f"{w_net_name(dl, a)} ({a.variant.upper()}) forward m={m} n={n} "
                            f"K={K} " + (f"B={B_global} global, {B}/GPU (strong scaling)"
                                         if strong else f"B={B}/GPU")
                            + f", all layers' Z/E/L/T written"
                            f"{'' if keep_all else ' (lean: last only)'} + fused per-layer "
                            f"{'L1L1' if a.variant == 'v4' else 'LASSO'} objective",
                "variant": a.variant, "m": m, "n": n, "layers": K, "batch_per_gpu": B,
                "path": path,
                "global_batch": w_global, "keep_all": keep_all,
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
        if world > 1:
            res["per_rank_kernel_ms"] = [k * 1e3 for k in kerns]
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
        if cfg2 is not None:
            f2 = (4 * K + 2) * m * n * 10000
            res["cfg2"] = {
                "workload": "BASELINE config 2: V4 forward m=256 n=512 K=15, B=10000 on one GPU, "
                            "all layers written + fused L1L1 objective",
                "value": cfg2["value"], "unit": "samples/s", "ms_per_step": cfg2["ms_per_step"],
                "kernel_ms": cfg2["kern"] * 1e3,
                "roofline_frac": f2 / cfg2["kern"] / PEAK_F32_MFMA,
                "path": {1: "fused", 5: "fused row-split"}.get(cfg2["path"], cfg2["path"]),
                "note": "path 5: 625 workgroups of 16 columns, each product's output rows split "
                        "over the 4 waves (the fused kernel's 64-column workgroups fill 157 of "
                        "the 256 CUs; DESIGN.md sections 12, 13.3b)",
                "objective_last_layer": cfg2["obj"],
            }
            if "split" in cfg2:
                sv, sms, sk, spath = cfg2["split"]
                res["cfg2"]["split_f16"] = {
                    "value": sv, "ms_per_step": sms, "kernel_ms": sk * 1e3,
                    "path": {4: "fused-split-f16"}.get(spath, spath),
                    "roofline_frac_f16_over_3": f2 / sk / (PEAK_BF16_MFMA / 3),
                    "note": "same workload, fp32 GEMMs as three exactly split f16 MFMA products "
                            "(the split_f16 line above; fp32 parity tolerances)"}
        for name, c in cfg45.items():
            m_, n_, K_, B_ = c["shape"]
            fl = (4 * K_ + 2) * m_ * n_ * B_
            pk = PEAK_BF16_MFMA if c["prec"] == "bf16" else PEAK_F32_MFMA
            res[name] = {
                "workload": (f"BASELINE config {name[-1]}: {c['var'].upper()} forward m={m_} "
                             f"n={n_} K={K_}, B={B_} on one GPU, "
                             f"{'bf16 MFMA operands / fp32 state' if c['prec'] == 'bf16' else 'fp32'}"
                             ", all layers written + fused objective" +
                             (f"; parameters: reference init except W = {c['wscale']} (A^T + "
                              "1e-3 N), which contracts (the reference's 0.4 diverges at this "
                              "shape: objective 2.3e27 at K=40)" if c["wscale"] else
                              "; reference-init parameters")),
                "value": c["value"], "unit": "samples/s", "ms_per_step": c["ms_per_step"],
                "path": {1: "fused", 2: "per-layer", 3: "bf16-tiles", 4: "fused-split-f16"}.get(
                    c["path"], c["path"]),
                "kernels_ms": c["kern"] * 1e3,
                "roofline_frac": fl / c["kern"] / pk,
                "roofline_peak": "bf16 dense MFMA" if c["prec"] == "bf16" else "fp32 MFMA",
                "objective_last_layer": c["obj"],
            }
        if v1 is not None:
            f1 = (4 * K + 2) * m * n * v1["B"]
            b1 = alg_bytes("v1", m, n, K, v1["B"], True)
            res["v1"] = {
                "workload": f"DLADMMNet (V1, main_lena.py:16-102) forward m={m} n={n} K={K}, "
                            f"B={v1['B']}/GPU, per-sample (m, B) beta1/beta2 per layer, every "
                            "layer's Z/E/L written (the reference's return lists); "
                            "reference-init parameters (betas 1, W = A^T + 1e-3 N)",
                "value": v1["value"], "unit": "samples/s", "ms_per_step": v1["ms_per_step"],
                "path": {1: "fused", 2: "per-layer"}.get(v1["path"], v1["path"]),
                "kernel": "dladmm::fused_kernel (one launch)",
                "kernel_ms": v1["kern"] * 1e3,
                "roofline_frac": f1 / v1["kern"] / PEAK_F32_MFMA,
                "roofline_peak": "fp32 MFMA 157.3 TF/s",
                "flop_per_launch": f1,
                "algorithmic_bytes_per_launch": b1,
                "bytes_per_sample": b1 / v1["B"],
                "hbm_frac_algorithmic": b1 / v1["kern"] / PEAK_HBM,
            }
            if "split" in v1:
                sv, sms, sk, spath = v1["split"]
                res["v1"]["split_f16"] = {
                    "value": sv, "ms_per_step": sms, "kernel_ms": sk * 1e3,
                    "path": {4: "fused-split-f16"}.get(spath, spath),
                    "roofline_frac_f16_over_3": f1 / sk / (PEAK_BF16_MFMA / 3),
                    "note": "same V1 workload, fp32 GEMMs as three exactly split f16 MFMA "
                            "products, the per-sample betas in the split kernel's epilogue "
                            "(fp32 parity tolerances)"}
        if cfg3 is not None:
            f3 = (4 * K + 2) * m * n * cfg3["B"]
            res["cfg3_strong"] = {
                "workload": f"BASELINE config 3: V4 forward m={m} n={n} K={K}, B=262144 global "
                            f"batch-sharded over {world} GPU(s) ({cfg3['B']}/GPU), all layers "
                            "written + fused L1L1 objective, one RCCL all-reduce of [K,2] sums",
                "scaling": "strong",
                "value": cfg3["value"],
                "unit": "samples/s",
                "ms_per_step": cfg3["ms_per_step"],
                "kernel_ms_max_over_ranks": cfg3["kern"] * 1e3,
                "per_rank_kernel_ms": [k * 1e3 for k in cfg3["kerns"]],
                "efficiency_within_run": (sum(cfg3["kerns"]) / world) / (cfg3["ms_per_step"]
                                                                         * 1e-3),
                "efficiency_note": "mean per-rank kernel time / wall time per step (1.0 = the "
                                   "step is all kernel; the driver computes scaling efficiency "
                                   "across N itself)",
                "roofline_frac": f3 / cfg3["kern"] / PEAK_F32_MFMA,
                "objective_last_layer": cfg3["obj"],
            }
        if train is not None:
            res["train"] = {k: train[k] for k in (
                "metric", "batch", "step_ms", "samples_per_s", "forward_ms", "backward_ms",
                "backward_tflops", "backward_frac_fp32_mfma", "loss_path", "split_f16",
                "ref_batch", "error")
                if k in train}
            res["train"]["note"] = ("V4 m=256 n=512 K=15 training step (zero_grad, forward with "
                                    "saved A Z_k, fused L1L1 objective with decay, reverse-sweep "
                                    "backward + split-K weight gradients, torch Adam); backward "
                                    "FLOP = 6 m n K B performed (tools/bench_train.py)")
        if world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(
                m, n, K, [int(x) for x in a.cpu_batch.split(",") if x], a.cpu_runs, a.variant)
        print(json.dumps(res), flush=True)
    if use_dist:
        dist.destroy_process_group()


def w_net_name(dl, a):
    return {"v4": dl.DLADMMNetScalar, "v6": dl.DLADMMNetLasso, "v1": dl.DLADMMNet}[a.variant].NAME


def alg_bytes(variant, m, n, K, B, keep_all):
    """Algorithmic HBM bytes of one forward launch: inputs X, Z0, E0, L0; outputs
    Z, E, L of every layer (keep_all) or of the last; T_0..T_K for the variants that return it
    (V4-V6; V1-V3 write none); V1's per-sample beta1 / beta2 of every layer (2 K m per sample);
    the weights (K + 1) m n once per launch.  V4 keep_all: 83,072 B/sample + 8 MiB; V1: 97,408
    at B = 65,536."""
    with_t = variant not in ("v1", "v2", "v3")
    io = (m + n + 2 * m) + (K if keep_all else 1) * (n + 2 * m)
    if with_t:
        io += (K + 1) * m if keep_all else m
    if variant == "v1":
        io += 2 * K * m
    return 4 * io * B + (K + 1) * m * n * 4


# ------------------------------------------------------------------------------------------------
# N-rank launch.  `python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment) starts N
# fresh rank processes through torch.distributed.run -- one per GPU, RCCL over xGMI -- from a
# parent that never touches the GPU (no HIP call, no torch.cuda initialisation: on this pool a
# process that initialised the GPU must not spawn-and-exec its replacement, and the ranks must own
# their devices).  The parent forwards rank 0's JSON line and exits with torch.distributed.run's
# status (non-zero if any rank failed).  Under an external launcher (the driver's
# `torch.distributed.run ... bench.py --gpus N`) WORLD_SIZE is set and must equal --gpus.
# Reference anchor: the only multi-GPU line of the reference is the commented-out
# `nn.DataParallel` (main_lena.py:192, main_syn_l1l1_scalar.py:238).

def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(argv, n, port, script=None):
    """(command, env) of the N-rank launch; pure host logic (tested on CPU)."""
    script = script or os.path.abspath(__file__)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
           script] + list(argv)
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this host driver
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return cmd, env


def world_check(gpus, environ=None):
    """None when the process should run as a rank (N = 1, or WORLD_SIZE set and equal to --gpus),
    "launch" when it should start the N ranks itself; raises SystemExit on a mismatch (a run that
    asked for N GPUs must never print a line measured on another count)."""
    environ = os.environ if environ is None else environ
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    ws = environ.get("WORLD_SIZE")
    if ws is None:
        return "launch" if gpus > 1 else None
    if int(ws) != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {gpus}: refusing to report an "
                         f"{ws}-rank measurement as {gpus} GPUs")
    return None


def visible_gpu_count(environ=None, kfd="/sys/class/kfd/kfd/topology/nodes", dri="/dev/dri"):
    """GPUs this process could use, counted WITHOUT any HIP or torch.cuda call (the launcher
    parent must not initialise the runtime: torch.cuda.device_count() falls back to
    hipGetDeviceCount when amdsmi is not importable).  The KFD topology lists one node per agent
    of the HOST (a container sees all of them); a GPU node has a non-zero simd_count and counts
    only if this process can open its render node, /dev/dri/renderD<drm_render_minor> -- what
    the ROCm runtime itself needs.  A *_VISIBLE_DEVICES list narrows the count the way the
    runtime applies it (ROCR first, then HIP / CUDA on top); a list that starts with an invalid
    id ("-1" hides every device) leaves none.  None when the topology is unreadable (no KFD
    driver: the ranks' own start-up then decides)."""
    environ = os.environ if environ is None else environ
    try:
        nodes = sorted(int(d) for d in os.listdir(kfd) if d.isdigit())
    except OSError:
        return None
    gpus = opened = 0
    for nd in nodes:
        try:
            props = open(os.path.join(kfd, str(nd), "properties")).read().split("\n")
        except OSError:
            continue
        kv = dict(ln.split() for ln in props if len(ln.split()) == 2)
        simd, minor = kv.get("simd_count", "0"), kv.get("drm_render_minor")
        if not (simd.isdigit() and int(simd) > 0):
            continue
        gpus += 1
        if minor is not None and os.access(os.path.join(dri, f"renderD{minor}"),
                                           os.R_OK | os.W_OK):
            opened += 1
    # no render node readable at all (no /dev/dri in this mount namespace): the check cannot
    # tell, so the topology's count stands rather than refusing every launch
    if opened:
        gpus = opened
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = environ.get(var)
        if not v:   # unset or empty: no narrowing (the ranks' own start-up decides)
            continue
        ids = [x.strip() for x in v.split(",") if x.strip() != ""]
        # the runtime stops at the first id it cannot parse ("-1" and the like): none before it
        valid = 0
        for x in ids:
            if not (x.isdigit() or x.startswith("GPU-")):
                break
            valid += 1
        gpus = min(gpus, valid)
    return gpus


def self_launch(argv, n) -> int:
    """Start n ranks (see above); print rank 0's JSON line; return the launcher's exit status."""
    import subprocess
    backend = os.environ.get("DLADMM_BENCH_BACKEND", "nccl")
    # DLADMM_KFD_TOPOLOGY points the count at another topology tree (the CPU tests' fake one);
    # the self-test ranks touch no device, so without it they skip the count
    topo = os.environ.get("DLADMM_KFD_TOPOLOGY")
    if backend == "nccl" and ("--launch-selftest" not in argv or topo):
        # from the KFD topology: no HIP call in this process (the CPU tests' fake tree carries
        # its render nodes in a dri/ directory beside the node directories)
        have = visible_gpu_count(kfd=topo, dri=os.path.join(topo, "dri")) \
            if topo else visible_gpu_count()
        if have is not None and have < n:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    cmd, env = launch_plan(argv, n, free_port())
    print("[bench.py] launching: " + " ".join(cmd), file=sys.stderr, flush=True)
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    js = [ln for ln in lines if ln.lstrip().startswith("{")]
    for ln in lines:
        if ln not in js:
            print(ln, file=sys.stderr)
    if p.returncode == 0 and len(js) != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {len(js)}", file=sys.stderr)
        return 3
    for ln in js:
        print(ln, flush=True)
    return p.returncode


def launch_selftest(a):
    """`--launch-selftest`: the rank side of the launcher with no device at all (gloo on CPU):
    each rank all-reduces its rank id; rank 0 prints one JSON line.  Exercises the real
    torch.distributed.run spawn, env and port plumbing in the CPU tests."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist.init_process_group("gloo")
    t = torch.tensor([float(rank)])
    dist.all_reduce(t)
    ranks = [torch.zeros(1) for _ in range(world)]
    dist.all_gather(ranks, torch.tensor([float(rank)]))
    if rank == 0:
        print(json.dumps({"n_gpus": world, "rank_sum": float(t[0]),
                          "ranks": [int(x) for x in ranks]}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    _argv = sys.argv[1:]
    _a = parse()
    if world_check(_a.gpus) == "launch":
        sys.exit(self_launch(_argv, _a.gpus))
    if _a.launch_selftest:
        launch_selftest(_a)
    else:
        main()
