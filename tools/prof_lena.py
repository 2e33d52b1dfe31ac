"""torch.profiler breakdown of one main_lena.py training step (V1, B = 20, the fused lena loss)
on the GPU: which kernels the small batch spends its time in.

    python tools/prof_lena.py [--batch 20]
"""
import argparse
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import bench_train  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=20)
    a = ap.parse_args()
    ta = bench_train.parser().parse_args(["--variant", "v1", "--lena-loss", "--lena-fused",
                                          "--batch", str(a.batch), "--steps", "5", "--warmup", "3"])
    bench_train.run(ta)   # warm
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as p:
        bench_train.run(ta)
        torch.cuda.synchronize()
    print(p.key_averages().table(sort_by="self_cuda_time_total", row_limit=20))


if __name__ == "__main__":
    main()
