#!/bin/bash
# A/B timing of fused-kernel builds (tools/ablate.py -> lib/abl/<name>/libdladmm_hip.so) against
# the in-tree library on the fp32 headline, ROUNDS times interleaved on one box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abl
ARGS=${BENCH_ARGS:---no-split --no-cpu-baseline --steps 20}
for round in $(seq 1 ${ROUNDS:-2}); do
  for L in d-ladmm_amd/lib/libdladmm_hip.so d-ladmm_amd/lib/abl/*/libdladmm_hip.so; do
    v=$(basename $(dirname $L))
    DLADMM_LIB=$L timeout -k 10 120 python bench.py $ARGS > gpurun_out/abl/$v.$round.json 2> gpurun_out/abl/$v.err || { echo "$v failed"; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abl/$v.$round.json').read().strip().splitlines()[-1]); print('$v', round(d['roofline']['kernel_ms'], 3), 'ms', round(d['value'] / 1e6, 2), 'M/s', round(d['roofline']['frac'], 4))"
  done
done
