#!/bin/bash
# Round 6, first GPU call: the whole GPU suite (parity margins logged), the default bench, an
# RCCL (nccl backend) rehearsal at world 1, and a rocprofv3 kernel summary of the V1 leg.
mkdir -p gpurun_out/r06
export DLADMM_PARITY_JSON=gpurun_out/r06/parity_log.json
tools/gpu_run.sh \
  "1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gputests.log 2>&1" \
  "600 python -u bench.py > gpurun_out/r06/bench.json 2> gpurun_out/r06/bench.err" \
  "300 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 DLADMM_BENCH_DIST=1 python -u bench.py --gpus 1 --no-cfg3 --no-train --no-cpu-baseline --steps 10 > gpurun_out/r06/rccl_world1.json 2> gpurun_out/r06/rccl_world1.err" \
  "300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/v1prof -o v1 -- python3 bench.py --variant v1 --no-cfg3 --no-train --no-cpu-baseline --no-split --steps 20 > gpurun_out/r06/v1_bench.json 2> gpurun_out/r06/v1_bench.err"
