#!/bin/bash
# kernel breakdown of the unchanged reference loop (V4, torch-op loss over Z_k: the GZ reverse)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04gz
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v4 -o run \
  -- python3 $R/tools/bench_train.py --variant v4 --steps 10 --warmup 2 > $O/v4.log 2>&1 || { echo failed; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v3 -o run \
  -- python3 $R/tools/bench_train.py --variant v3 --fused-loss --steps 10 --warmup 2 > $O/v3.log 2>&1 || { echo failed; exit 1; }
echo done
