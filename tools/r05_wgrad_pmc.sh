#!/bin/bash
# Round 5: rocprofv3 counter passes over the split-f16 training step (tools/bench_train.py
# --precision f32_split, V4 256 x 512 K=15 B=65,536), for the weight-gradient kernel
# (python tools/pmc_table.py gpurun_out/prof_wx3 wgrad_x3).  One run per pass, each under its
# own timeout.  Output: gpurun_out/prof_wx3/p<i>/.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof_wx3
run() {
  name=$1; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv \
    -d $R/gpurun_out/prof_wx3/$name -o run -- python3 $R/tools/bench_train.py --variant v4 \
    --fused-loss --precision f32_split --steps 2 --warmup 1 > $R/gpurun_out/prof_wx3/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run p2 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_MISC
run p3 FETCH_SIZE
