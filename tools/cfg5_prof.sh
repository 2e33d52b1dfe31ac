#!/bin/bash
# rocprofv3 kernel trace + stats of the config-5 bf16 bench (both tile widths)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
for t in narrow wide; do
  DLADMM_BF16_TILE=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/cfg5prof/$t -o run -- python3 $R/bench.py --precision bf16 --m 1024 --n 4096 --batch 16384 --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/cfg5prof/$t.log 2>&1 || exit 1
done
