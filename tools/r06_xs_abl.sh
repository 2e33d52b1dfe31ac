#!/bin/bash
# Round 6: where path 6's time goes -- timing-only builds without the hand-off poll (xs1), also
# without the exchange loads (xs3), also without the exchange stores (xs7).
mkdir -p gpurun_out/r06z
tools/gpu_run.sh \
  "300 python -u tools/bench_fwd_ab.py --libs main,d-ladmm_amd/lib/abl/xs1/libdladmm_hip.so,d-ladmm_amd/lib/abl/xs3/libdladmm_hip.so,d-ladmm_amd/lib/abl/xs7/libdladmm_hip.so --batches 20,1000 --reps 10 > gpurun_out/r06z/abl.json 2> gpurun_out/r06z/abl.err" \
  "120 python -u tools/xs_smoke.py > gpurun_out/r06z/smoke.txt 2>&1"
