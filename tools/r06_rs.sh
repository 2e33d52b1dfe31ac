#!/bin/bash
# Round 6: path 5 (small-batch row-split fused forward).  Its own tests (bit-equal to path 1,
# oracle, plan scope), then the suites that now run small batches through it, then timing.
mkdir -p gpurun_out/r06j
tools/gpu_run.sh \
  "300 python -u -m pytest tests/test_gpu_rowsplit.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06j/rs_tests.log 2>&1" \
  "900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lskm.py tests/test_gpu_eval.py tests/test_gpu_graph.py tests/test_gpu_poison.py tests/test_gpu_configs.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06j/tests.log 2>&1" \
  "600 python -u tools/bench_eval.py --reps 3 --ab > gpurun_out/r06j/eval.json 2> gpurun_out/r06j/eval.err"
