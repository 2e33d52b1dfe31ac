#!/bin/bash
# backward alone (tools/bench_bwd.py, V4 256x512 K=15 B=65536 fused objective): kernel stats
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04bp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run \
  -- python3 $R/tools/bench_bwd.py --reps 10 > $O/bwd.log 2>&1 || { echo failed; exit 1; }
tail -1 $O/bwd.log
echo done
