#!/bin/bash
# PMC passes over a short split-f16 bench run (one rocprofv3 run per counter set).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/prof/counters.txt 2>&1
B="$R/bench.py --precision ${PREC:-f32_split} --no-cpu-baseline --steps 5 --warmup 1"
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/gpurun_out/prof/p$i -o run -- python3 $B > $R/gpurun_out/prof/p$i.log 2>&1
  echo "pass $i ($set) rc=$?"
done << 'SETS'
SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES
SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS
SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS
SETS
