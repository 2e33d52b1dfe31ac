#!/bin/bash
# Round 6: the row-split lena objective with one workgroup per (16-column group, layer): the lena /
# training tests, main_lena's B = 20 step and its kernel breakdown.
mkdir -p gpurun_out/r06ll
tools/gpu_run.sh \
  "600 python -u -m pytest tests/test_gpu_lena.py tests/test_gpu_training.py tests/test_capi.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06ll/tests.log 2>&1" \
  "300 python -u tools/bench_train.py --batch 20 --steps 50 --warmup 5 --variant v1 --lena-loss --lena-fused > gpurun_out/r06ll/v1_b20_lena.json 2> gpurun_out/r06ll/v1_b20_lena.err" \
  "300 python -u tools/prof_lena.py > gpurun_out/r06ll/prof_lena.txt 2>&1"
