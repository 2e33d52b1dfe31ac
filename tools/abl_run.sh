#!/bin/bash
# timing ablations of the fused kernel (tools/ablate.py builds the variants)
args=()
for v in "${@:-base}"; do
  if [ $v = base ]; then L=""; else L="DLADMM_LIB=d-ladmm_amd/lib/abl/$v/libdladmm_hip.so"; fi
  args+=("120 $L python bench.py --no-cpu-baseline --steps 10 ${ABL_ARGS} > gpurun_out/abl_$v.log 2>&1")
done
exec tools/gpu_run.sh "${args[@]}"
