#!/bin/bash
# Round 6, library with path 6 (four-workgroup row split) and the V1 / cotangent row-split reverse
# sweep (bwd paths 2 and 3): the whole GPU suite (parity margins to r06v/parity_log.json), smoke(), the default bench.
mkdir -p gpurun_out/r06fin2
export DLADMM_PARITY_JSON=gpurun_out/r06fin2/parity_log.json
tools/gpu_run.sh \
  "1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06fin2/tests.log 2>&1" \
  "300 python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")' > gpurun_out/r06fin2/smoke.log 2>&1" \
  "600 python -u bench.py > gpurun_out/r06fin2/bench.json 2> gpurun_out/r06fin2/bench.err"
