#!/bin/bash
# training-step A/B: in-tree library vs lib/abl/*/ builds, interleaved rounds on one box
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/tab
for round in 1 2; do
  for L in d-ladmm_amd/lib/libdladmm_hip.so d-ladmm_amd/lib/abl/*/libdladmm_hip.so; do
    v=$(basename $(dirname $L))
    DLADMM_LIB=$L timeout -k 10 200 python tools/bench_train.py --fused-loss > gpurun_out/tab/$v.$round.json 2> gpurun_out/tab/$v.err || { echo "$v failed"; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/tab/$v.$round.json').read().strip().splitlines()[-1]); print('$v', round(d['step_ms'], 3), 'step ms', round(d['backward_ms'], 3), 'bwd ms')"
  done
done
