#!/bin/bash
# Round 6 counters (one rocprofv3 pass per counter set, each its own run):
#   cfg5  BASELINE config 5 (bf16 tiles, m=1024 n=4096 K=15 B=16384): MFMA-side counters that
#         are physical -- instruction and MOPS counts beside the busy-cycle counter (round 5's
#         SQ_VALU_MFMA_BUSY_CYCLES read 2^27 in every pass) and the derived MfmaUtil;
#   head  the fp32 headline (V4 B=65,536, fused kernel): the same counters on a kernel whose
#         MFMA rate is known from its FLOP / time (the validation of the counters);
#   cfg2  config 2 (V4 B=10,000): CU occupancy of the full fused kernel (the packing argument).
# -> gpurun_out/r06pmc/<workload>_<pass>/ ; python tools/r06_pmc_table.py
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r06pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C5="--precision bf16 --m 1024 --n 4096 --batch 16384 --steps 3 --warmup 1 --no-cpu-baseline"
HD="--no-cfg3 --no-train --no-cpu-baseline --no-split --steps 3 --warmup 1"
C2="--batch 10000 --no-cfg3 --no-train --no-cpu-baseline --no-split --steps 3 --warmup 1"
PA="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
PB="MfmaUtil"
PC="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
run() {  # workload, pass tag, counters
  local wl=$1 tag=$2; shift 2
  case $wl in head) A=$HD ;; cfg5) A=$C5 ;; cfg2) A=$C2 ;; esac
  echo "[r06_pmc] $wl $tag: $*"
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $O/${wl}_$tag \
    -o run -- python3 $R/bench.py $A > $O/${wl}_$tag.log 2>&1
}
for wl in head cfg5 cfg2; do
  run $wl pa $PA || { echo "fail $wl pa"; exit 1; }
  run $wl pc $PC || { echo "fail $wl pc"; exit 1; }
done
# the derived metric last (a counter name rocprofv3 may not take in --pmc)
for wl in head cfg5; do
  run $wl pb $PB || { echo "fail $wl pb (derived metric)"; exit 1; }
done
echo pmc done
