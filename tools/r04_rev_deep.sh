#!/bin/bash
# Round 4: DEEP operand prefetch in the reverse sweep -- equivalence tests, then an interleaved
# A/B of the backward against the previous build (d-ladmm_amd/lib/abl/r4a).  Logs in gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_reverse.py tests/test_gpu_backward.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_deep_tests.log 2>&1 \
  || { tail -30 gpurun_out/r04_deep_tests.log; exit 1; }
tail -1 gpurun_out/r04_deep_tests.log
timeout -k 10 300 python tools/bench_bwd.py --reps 10 \
  --libs main,d-ladmm_amd/lib/abl/r4a/libdladmm_hip.so > gpurun_out/r04_deep_ab.json || exit 1
cat gpurun_out/r04_deep_ab.json
