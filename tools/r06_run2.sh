#!/bin/bash
# Round 6, second GPU call: the whole GPU suite again (plan flags carried into autograd
# backwards) with the parity-margin log, and the list of PMC counters this rocprofv3 offers.
mkdir -p gpurun_out/r06b
export DLADMM_PARITY_JSON=gpurun_out/r06b/parity_log.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
tools/gpu_run.sh \
  "1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06b/gputests.log 2>&1" \
  "120 rocprofv3 -L > gpurun_out/r06b/counters.txt 2>&1"
