#!/bin/bash
# Round 6: path 6 with each pass's first weight fragments fetched during the hand-off before it:
# second pass: the fetch placed after the exchange loads (late), read-ahead 12; bit-equality.
mkdir -p gpurun_out/r06q
tools/gpu_run.sh \
  "120 python -u tools/xs_smoke.py > gpurun_out/r06q/smoke.txt 2>&1" \
  "300 python -u tools/bench_fwd_ab.py --libs main,d-ladmm_amd/lib/abl/late/libdladmm_hip.so,d-ladmm_amd/lib/abl/late12/libdladmm_hip.so,d-ladmm_amd/lib/abl/pf12/libdladmm_hip.so --batches 20,1000 --reps 10 > gpurun_out/r06q/abl.json 2> gpurun_out/r06q/abl.err"
