#!/bin/bash
# rocprofv3 passes over a short bench run (run on the GPU box from the repo root):
#   1. kernel trace + stats        -> gpurun_out/prof/kt
#   2. PMC pass: FETCH_SIZE        -> gpurun_out/prof/pmc_fetch
#   3. PMC pass: WRITE_SIZE        -> gpurun_out/prof/pmc_write
#   4. PMC pass: MFMA/VALU busy + GRBM_GUI_ACTIVE (clock) -> gpurun_out/prof/pmc_sq
# Each pass has its own time limit; the script stops at the first failing pass.
# The profiled bench runs the headline workload alone (--no-cfg3 --no-split: bench.py's default
# line also launches the same fused kernel for configs 2 and 3, which would mix three grid sizes
# into rocprofv3's per-kernel-name --stats average); BENCH_ARGS replaces that selection.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
BENCH="$R/bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline ${BENCH_ARGS---no-cfg3 --no-split}"
run() {
  local name=$1; shift
  echo "[profile] $name" | tee -a $OUT/steps.log
  timeout -k 10 400 rocprofv3 "$@" --output-format csv -d $OUT/$name -o run -- python3 $BENCH > $OUT/$name.log 2>&1
  local rc=$?
  echo "[profile] $name rc=$rc" | tee -a $OUT/steps.log
  return $rc
}
run kt --kernel-trace --stats || exit 1
run pmc_fetch --kernel-trace --pmc FETCH_SIZE || exit 1
run pmc_write --kernel-trace --pmc WRITE_SIZE || exit 1
run pmc_sq --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
exit 0
