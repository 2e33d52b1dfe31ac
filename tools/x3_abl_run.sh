#!/bin/bash
# GPU side of tools/x3_ablate.py: bench every built variant (lib/abl/*.so) and the in-tree
# library on the split-f16 path; one JSON line per variant in gpurun_out/abl/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abl
ARGS=${BENCH_ARGS:---precision f32_split --no-cpu-baseline --steps 10}
for L in d-ladmm_amd/lib/libdladmm_hip.so d-ladmm_amd/lib/abl/*.so; do
  v=$(basename $L .so)
  DLADMM_LIB=$L timeout -k 10 120 python bench.py $ARGS > gpurun_out/abl/$v.json 2> gpurun_out/abl/$v.err || { echo "$v failed"; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/abl/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['roofline']['kernel_ms'], 3), 'ms', round(d['value'] / 1e6, 2), 'M/s')"
done
