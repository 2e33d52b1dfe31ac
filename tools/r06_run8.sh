#!/bin/bash
# Round 6, library with path 5 (training forwards, V1, three per CU): the whole GPU suite (parity margins to r06r/parity_log.json), smoke(),
# the default bench.
mkdir -p gpurun_out/r06r
export DLADMM_PARITY_JSON=gpurun_out/r06r/parity_log.json
tools/gpu_run.sh \
  "1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06r/tests.log 2>&1" \
  "300 python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")' > gpurun_out/r06r/smoke.log 2>&1" \
  "600 python -u bench.py > gpurun_out/r06r/bench.json 2> gpurun_out/r06r/bench.err" \
  "600 python -u tools/bench_eval.py --reps 3 --ab > gpurun_out/r06r/eval.json 2> gpurun_out/r06r/eval.err"
