#!/bin/bash
# Round 6: the row-split form of the fused main_lena objective (dladmm_lena_f32 at small
# batches): its tests, main_lena's B = 20 training step and its kernel breakdown.
mkdir -p gpurun_out/r06t
tools/gpu_run.sh \
  "600 python -u -m pytest tests/test_gpu_lena.py tests/test_gpu_rowsplit.py tests/test_gpu_training.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06t/tests.log 2>&1" \
  "300 python -u tools/bench_train.py --batch 20 --steps 50 --warmup 5 --variant v1 --lena-loss --lena-fused > gpurun_out/r06t/v1_b20_lena.json 2> gpurun_out/r06t/v1_b20_lena.err" \
  "300 python -u tools/prof_lena.py > gpurun_out/r06t/prof_lena.txt 2>&1"
