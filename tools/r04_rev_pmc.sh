#!/bin/bash
# Round 4: rocprofv3 counter passes over the reverse-sweep backward (tools/bench_bwd.py, V4
# 256 x 512 K=15 B=65,536, fused objective).  One run per pass (gpurun rule), each under its own
# timeout.  Output: gpurun_out/prof_rev/p<i>/.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof_rev
run() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" --output-format csv \
    -d $R/gpurun_out/prof_rev/$name -o run -- python3 $R/tools/bench_bwd.py --reps 2 \
    > $R/gpurun_out/prof_rev/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run p2 SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INSTS_VALU SQ_INSTS_MFMA TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES
run p3 TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES
