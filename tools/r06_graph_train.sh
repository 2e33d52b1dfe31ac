#!/bin/bash
# Round 6: the reference loops' training steps replayed from one HIP graph (the step without the
# Python / launch overhead) beside the eager step: V4 at the l1l1 loop's B = 25 first, then V1
# with main_lena's fused objective at B = 20.
mkdir -p gpurun_out/r06gr2
tools/gpu_run.sh \
  "300 python -u tools/bench_train.py --batch 25 --steps 50 --warmup 5 --fused-loss --graph > gpurun_out/r06gr2/v4_b25_fused_graph.json 2> gpurun_out/r06gr2/v4_b25_fused_graph.err" \
  "300 python -u tools/bench_train.py --batch 20 --steps 50 --warmup 5 --variant v1 --lena-fused --graph > gpurun_out/r06gr2/v1_b20_lena_graph.json 2> gpurun_out/r06gr2/v1_b20_lena_graph.err"
