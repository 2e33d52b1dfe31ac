#!/bin/bash
# Round 4: reverse-ring A/B (4 slots = main, 6 slots, 6 slots + deep prefetch), then the list of
# PMC counters rocprofv3 offers on this GPU (for the reverse-kernel counter passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_bwd.py --reps 10 \
  --libs main,d-ladmm_amd/lib/abl/s6/libdladmm_hip.so,d-ladmm_amd/lib/abl/d6/libdladmm_hip.so \
  > gpurun_out/r04_slots_ab.json || exit 1
cat gpurun_out/r04_slots_ab.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 90 rocprofv3 -L > $R/gpurun_out/r04_avail.txt 2>&1
echo "avail rc=$?"
