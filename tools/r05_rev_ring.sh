#!/bin/bash
# Round 5: reverse-sweep weight-ring geometry, A/B in one process (tools/bench_bwd.py): 32-fragment
# chunks in 3 slots (half the ring barriers), 5 and 3 slots of 16 -> gpurun_out/r05_rev_ring.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
L=""
for v in rcf32 rs5 rs3; do L="$L,d-ladmm_amd/lib/abl/$v/libdladmm_hip.so"; done
timeout -k 10 400 python tools/bench_bwd.py --reps 10 --libs main$L > gpurun_out/r05_rev_ring.json || exit 1
cat gpurun_out/r05_rev_ring.json
