#!/bin/bash
# A/B of the slice-GEMM kernels (config 4 per-layer forward, training step) for the in-tree
# library and lib/abl/*/libdladmm_hip.so, ROUNDS times interleaved on one box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abl
for round in $(seq 1 ${ROUNDS:-2}); do
  for L in d-ladmm_amd/lib/libdladmm_hip.so d-ladmm_amd/lib/abl/*/libdladmm_hip.so; do
    v=$(basename $(dirname $L))
    DLADMM_LIB=$L timeout -k 10 200 python bench.py --variant v6 --m 512 --n 2048 --layers 40 --no-split --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/abl/c4_$v.$round.json 2> gpurun_out/abl/c4_$v.err || { echo "$v c4 failed"; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abl/c4_$v.$round.json').read().strip().splitlines()[-1]); print('cfg4 $v', round(d['ms_per_step'], 3), 'ms', round(d['value'] / 1e6, 3), 'M/s')"
    DLADMM_LIB=$L timeout -k 10 200 python tools/bench_train.py > gpurun_out/abl/tr_$v.$round.json 2> gpurun_out/abl/tr_$v.err || { echo "$v train failed"; exit 1; }
    echo "train $v $(tail -1 gpurun_out/abl/tr_$v.$round.json | cut -c1-300)"
  done
done
