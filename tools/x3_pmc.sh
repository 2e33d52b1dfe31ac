#!/bin/bash
# PMC passes over a short bench run of one kernel path (one rocprofv3 run per counter set,
# each under its own time limit; stops at the first failing pass).  Summarise with
#   python tools/pmc_table.py gpurun_out/prof <kernel-name-substring>
# PREC selects the bench precision (f32_split: dladmm::fused_x3_kernel; f32: fused_kernel).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --precision ${PREC:-f32_split} --no-split --no-cpu-baseline --steps 5 --warmup 1"
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/gpurun_out/prof/p$i -o run -- python3 $B > $R/gpurun_out/prof/p$i.log 2>&1
  rc=$?
  echo "pass $i ($set) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done << 'SETS'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_BARRIER SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM
TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA
FETCH_SIZE
WRITE_SIZE
SETS
