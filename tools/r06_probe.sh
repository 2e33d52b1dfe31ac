#!/bin/bash
# Round 6: the one-wave-per-SIMD 256 x 256 bf16 main-loop probe (tools/probe/bf16_tile256.hip)
# beside hipBLASLt on config 5's two products (tools/probe_gemm_ref.py).
mkdir -p gpurun_out/r06probe
tools/gpu_run.sh \
  "120 tools/probe/bf16_tile256 > gpurun_out/r06probe/tile256.jsonl 2> gpurun_out/r06probe/tile256.err" \
  "240 python -u tools/probe_gemm_ref.py > gpurun_out/r06probe/hipblaslt.json 2> gpurun_out/r06probe/hipblaslt.err"
