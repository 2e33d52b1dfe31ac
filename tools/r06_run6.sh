#!/bin/bash
# Round 6: V1 on the split-f16 kernel -- the split / backward / lena / config suites, then the
# default bench (its v1 line carries the split leg).
mkdir -p gpurun_out/r06c
export DLADMM_PARITY_JSON=gpurun_out/r06c/parity_log.json
tools/gpu_run.sh \
  "900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_backward.py tests/test_gpu_lena.py tests/test_gpu_configs.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06c/tests.log 2>&1" \
  "600 python -u bench.py > gpurun_out/r06c/bench.json 2> gpurun_out/r06c/bench.err"
