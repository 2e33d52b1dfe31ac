#!/bin/bash
# Timing of the reverse-kernel ablation builds (tools/ablate_units.py, REV_ABL bits; WRONG
# results by design): backward ms of the fused-loss training step per variant.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/revabl
for v in ${VARIANTS:-ra0 ra2 ra4 ra6 ra24 ra32 ra96}; do
  DLADMM_LIB=d-ladmm_amd/lib/abl/$v/libdladmm_hip.so timeout -k 10 120 python tools/bench_train.py --fused-loss --steps 5 --warmup 1 > gpurun_out/revabl/$v.json 2> gpurun_out/revabl/$v.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/revabl/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['backward_ms'],3))"
done
