#!/bin/bash
# GPU side of `tools/ablate.py --unit dladmm_tile_bf16.hip ...`: the config-5 bf16 bench for the
# in-tree library and every built variant (lib/abl/*/libdladmm_hip.so), ROUNDS times interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/tabl
ARGS=${BENCH_ARGS:---precision bf16 --m 1024 --n 4096 --batch 16384 --steps 10 --warmup 2 --no-cpu-baseline}
for round in $(seq 1 ${ROUNDS:-2}); do
  for L in d-ladmm_amd/lib/libdladmm_hip.so d-ladmm_amd/lib/abl/*/libdladmm_hip.so; do
    v=$(basename $(dirname $L))
    DLADMM_LIB=$L timeout -k 10 120 python bench.py $ARGS > gpurun_out/tabl/$v.$round.json 2> gpurun_out/tabl/$v.err || { echo "$v failed"; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/tabl/$v.$round.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'], 3), 'ms', round(d['value'] / 1e6, 3), 'M/s')"
  done
done
