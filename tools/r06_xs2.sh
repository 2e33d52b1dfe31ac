#!/bin/bash
# Round 6: path 6 after the objective-slot fix: smoke, the row-split / capi / training / lena /
# lskm / eval suites, the V4 B = 25 training step.
mkdir -p gpurun_out/r06y
tools/gpu_run.sh \
  "120 python -u tools/xs_smoke.py > gpurun_out/r06y/smoke.txt 2>&1" \
  "900 python -u -m pytest tests/test_gpu_rowsplit.py tests/test_capi.py tests/test_gpu_training.py tests/test_gpu_lena.py tests/test_gpu_lskm.py tests/test_gpu_eval.py tests/test_gpu_configs.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06y/tests.log 2>&1" \
  "300 python -u tools/bench_train.py --batch 25 --steps 50 --warmup 5 --variant v4 --fused-loss > gpurun_out/r06y/v4_b25_fused.json 2> gpurun_out/r06y/v4_b25_fused.err" \
  "300 python -u tools/prof_lena.py > gpurun_out/r06y/prof_lena.txt 2>&1"
