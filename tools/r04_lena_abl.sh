#!/bin/bash
# lena kernel alone, full build and the LENA_ABL timing variants (tools/ablate.py builds)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/r04la
for v in ${LVARS:-base l2 l16 l32}; do
  if [ $v = base ]; then lib=""; else lib=$R/d-ladmm_amd/lib/abl/$v/libdladmm_hip.so; fi
  DLADMM_LIB=$lib timeout -k 10 120 python tools/bench_lena.py > gpurun_out/r04la/$v.json || { echo "$v failed"; exit 1; }
  echo "$v $(cat gpurun_out/r04la/$v.json)"
done
