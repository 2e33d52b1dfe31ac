#!/bin/bash
# Round 6: the row-split reverse sweep widened to V1 and E / L / T cotangents (bwd path 2 for
# main_lena's training step): its tests, the backward suites it now serves, main_lena's B = 20
# step and its kernel breakdown.
mkdir -p gpurun_out/r06u
tools/gpu_run.sh \
  "900 python -u -m pytest tests/test_gpu_rowsplit.py tests/test_gpu_lena.py tests/test_gpu_training.py tests/test_gpu_backward.py tests/test_gpu_reverse.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06u/tests.log 2>&1" \
  "300 python -u tools/bench_train.py --batch 20 --steps 50 --warmup 5 --variant v1 --lena-loss --lena-fused > gpurun_out/r06u/v1_b20_lena.json 2> gpurun_out/r06u/v1_b20_lena.err" \
  "300 python -u tools/prof_lena.py > gpurun_out/r06u/prof_lena.txt 2>&1"
