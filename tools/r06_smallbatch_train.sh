#!/bin/bash
# Round 6: the reference's own training batch sizes (main_syn_l1l1_scalar.py -bs 25,
# main_lena.py batch_size = 20): one training step's time, fused and torch-op losses, and the
# CPU reference restatement's step for comparison (tools/bench_train.py).
mkdir -p gpurun_out/r06m
tools/gpu_run.sh \
  "300 python -u tools/bench_train.py --batch 25 --steps 50 --warmup 5 > gpurun_out/r06m/v4_b25.json 2> gpurun_out/r06m/v4_b25.err" \
  "300 python -u tools/bench_train.py --batch 25 --steps 50 --warmup 5 --fused-loss > gpurun_out/r06m/v4_b25_fused.json 2> gpurun_out/r06m/v4_b25_fused.err" \
  "300 python -u tools/bench_train.py --batch 20 --steps 50 --warmup 5 --variant v1 --lena-loss --lena-fused > gpurun_out/r06m/v1_b20_lena.json 2> gpurun_out/r06m/v1_b20_lena.err"
