#!/bin/bash
# Round 6: rocprofv3 kernel statistics of the small-batch paths (B = 20, V4 K = 15, fused
# objective): forward paths 6 / 5 / 1 and backward paths 3 / 2 / 1, interleaved in one process.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06xp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06xp/fwd -o fwd -- python3 tools/bench_fwd_ab.py --batches 20 --flag-set 0,128,64 --reps 5 > gpurun_out/r06xp/fwd.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06xp/bwd -o bwd -- python3 tools/bench_bwd.py --batch 20 --flag-set 0,128,64 --reps 5 > gpurun_out/r06xp/bwd.log 2>&1
