#!/bin/bash
# Round 5: L2 hit rate and HBM requests of the queue launch at 1 / 2 / 4 lag classes against the
# one-phase wide tiles (config 5) -> gpurun_out/qpmc/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/qpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="--precision bf16 --m 1024 --n 4096 --batch 16384 --no-cpu-baseline --steps 3 --warmup 1"
for mode in "0 1" "1 1" "1 2" "1 4"; do
  set -- $mode
  DLADMM_BF16_TILE=wide DLADMM_BF16_QUEUE=$1 DLADMM_BF16_QUEUE_LAGS=$2 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/q$1_$2 -o run -- python3 $R/bench.py $B > $O/q$1_$2.log 2>&1 || exit 1
done
echo pmc done
