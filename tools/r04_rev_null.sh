#!/bin/bash
# Reverse-sweep operand-traffic ablations (REV_ABL 128..2048: one G2' operand through a null
# buffer view -- instructions kept, memory traffic gone; WRONG results by design), A/B in one
# process with tools/bench_bwd.py.  Output: gpurun_out/r04_rev_null.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
L=""
for v in r0 r128 r256 r512 r1024 r2048 r3968; do L="$L,d-ladmm_amd/lib/abl/$v/libdladmm_hip.so"; done
timeout -k 10 400 python tools/bench_bwd.py --reps 10 --libs main$L > gpurun_out/r04_rev_null.json || exit 1
cat gpurun_out/r04_rev_null.json
