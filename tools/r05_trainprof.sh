#!/bin/bash
# Kernel-level breakdown of the training steps per variant (rocprofv3 --kernel-trace --stats),
# fused loss, B = 65,536: gpurun_out/r05t/<variant>/run_kernel_stats.csv
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-v1 v4}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run \
    -- python3 $R/tools/bench_train.py --variant $v --fused-loss --steps 10 --warmup 2 \
    > $O/$v.log 2>&1 || { echo "$v failed"; exit 1; }
  grep '"step_ms"' $O/$v.log | tail -1 | cut -c1-300
done
echo done
