#!/bin/bash
# split-f16 forward A/B: in-tree library vs lib/abl/*/ builds, interleaved rounds on one box
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sab
for round in 1 2 3; do
  for L in d-ladmm_amd/lib/libdladmm_hip.so d-ladmm_amd/lib/abl/*/libdladmm_hip.so; do
    v=$(basename $(dirname $L))
    DLADMM_LIB=$L timeout -k 10 120 python bench.py --precision f32_split --no-cpu-baseline --steps 20 > gpurun_out/sab/$v.$round.json 2> gpurun_out/sab/$v.err || { echo "$v failed"; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/sab/$v.$round.json').read().strip().splitlines()[-1]); print('$v', round(d['roofline']['kernel_ms'], 4), 'ms', round(d['value'] / 1e6, 2), 'M/s')"
  done
done
