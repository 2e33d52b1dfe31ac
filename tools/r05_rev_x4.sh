#!/bin/bash
# Round 5: would fragment-order dwordx4 operand loads pay in the reverse sweep?  Timing-only
# ablation builds (REV_ABL 4096 X, 8192 P, 16384 adjoint of E, 28672 all three: one dwordx4 per
# G2' block instead of a dword per row; WRONG results), A/B in one process (tools/bench_bwd.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
L=""
for v in r0 rx4 rp4 rae4 rall4; do L="$L,d-ladmm_amd/lib/abl/$v/libdladmm_hip.so"; done
timeout -k 10 400 python tools/bench_bwd.py --reps 10 --libs main$L > gpurun_out/r05_rev_x4.json || exit 1
cat gpurun_out/r05_rev_x4.json
