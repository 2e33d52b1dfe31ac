#!/bin/bash
# Config-5 (bf16, m=1024 n=4096 K=15 B=16384) HBM traffic: a kernel-trace + stats pass, then one
# rocprofv3 PMC pass per TCC counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass).
#   tools/cfg5_pmc.sh  -> gpurun_out/cfg5pmc/p{1,2,3}/ ; python tools/cfg5_pmc_table.py
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/cfg5pmc
mkdir -p $O
B="--precision bf16 --m 1024 --n 4096 --batch 16384 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p1 -o run \
  -- python3 $R/bench.py $B > $O/p1.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/p2 -o run \
  -- python3 $R/bench.py $B > $O/p2.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/p3 -o run \
  -- python3 $R/bench.py $B > $O/p3.log 2>&1 || exit 1
