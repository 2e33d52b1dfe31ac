#!/bin/bash
# Round 6: bwd path 3 after the parameter-slot bar fix: the row-split / reverse / backward suites,
# and the backward A/B (bwd paths 3 / 2 / 1 in one process) at the reference loops' batches.
mkdir -p gpurun_out/r06bb
tools/gpu_run.sh \
  "900 python -u -m pytest tests/test_gpu_rowsplit.py tests/test_capi.py tests/test_gpu_reverse.py tests/test_gpu_backward.py tests/test_gpu_training.py tests/test_gpu_lena.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06bb/tests.log 2>&1" \
  "300 python -u tools/bench_bwd.py --batch 25 --flag-set 0,128,64 --reps 10 > gpurun_out/r06bb/bwd_b25.json 2> gpurun_out/r06bb/bwd_b25.err" \
  "300 python -u tools/bench_bwd.py --batch 25 --gz --flag-set 0,128,64 --reps 10 > gpurun_out/r06bb/bwd_b25_gz.json 2> gpurun_out/r06bb/bwd_b25_gz.err" \
  "300 python -u tools/bench_bwd.py --batch 1000 --flag-set 0,128,64 --reps 10 > gpurun_out/r06bb/bwd_b1000.json 2> gpurun_out/r06bb/bwd_b1000.err"
