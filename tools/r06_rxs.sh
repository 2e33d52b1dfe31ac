#!/bin/bash
# Round 6: bwd path 3, the reverse sweep over four workgroups per 16 columns (after path 6):
# the backward suites, the reference loops' training steps and a kernel breakdown.
mkdir -p gpurun_out/r06b
tools/gpu_run.sh \
  "900 python -u -m pytest tests/test_gpu_rowsplit.py tests/test_capi.py tests/test_gpu_reverse.py tests/test_gpu_backward.py tests/test_gpu_training.py tests/test_gpu_lena.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06b/tests.log 2>&1" \
  "300 python -u tools/bench_train.py --batch 20 --steps 50 --warmup 5 --variant v1 --lena-loss --lena-fused > gpurun_out/r06b/v1_b20_lena.json 2> gpurun_out/r06b/v1_b20_lena.err" \
  "300 python -u tools/bench_train.py --batch 25 --steps 50 --warmup 5 --fused-loss > gpurun_out/r06b/v4_b25_fused.json 2> gpurun_out/r06b/v4_b25_fused.err" \
  "300 python -u tools/prof_lena.py > gpurun_out/r06b/prof_lena.txt 2>&1"
