#!/bin/bash
# GPU side of tools/x3_ablate.py: bench every built variant (lib/abl/*.so) and the in-tree
# library on the split-f16 path, ROUNDS times interleaved (same box: A/B comparisons only hold
# within one call); one JSON line per variant and round in gpurun_out/abl/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abl
ARGS=${BENCH_ARGS:---precision f32_split --no-split --no-cpu-baseline --steps 20}
for round in $(seq 1 ${ROUNDS:-2}); do
  for L in d-ladmm_amd/lib/libdladmm_hip.so d-ladmm_amd/lib/abl/*.so; do
    v=$(basename $L .so)
    DLADMM_LIB=$L timeout -k 10 120 python bench.py $ARGS > gpurun_out/abl/$v.$round.json 2> gpurun_out/abl/$v.err || { echo "$v failed"; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abl/$v.$round.json').read().strip().splitlines()[-1]); print('$v', round(d['roofline']['kernel_ms'], 3), 'ms', round(d['value'] / 1e6, 2), 'M/s')"
  done
done
