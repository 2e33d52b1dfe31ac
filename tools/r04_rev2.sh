#!/bin/bash
# Round 4: the reverse sweep for every variant (V1 / V2 / V3 / V4 / V5 / V6) -- the reverse
# tests (bit-equal to the per-layer backward), the backward and training tests, then training
# steps on both backward paths.  Logs in gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_reverse.py tests/test_gpu_backward.py \
  tests/test_gpu_training.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r04_rev2_tests.log 2>&1 || { tail -40 gpurun_out/r04_rev2_tests.log; exit 1; }
tail -1 gpurun_out/r04_rev2_tests.log
: > gpurun_out/r04_train2.jsonl
for spec in "v2 --fused-loss" "v3 --fused-loss" "v4 --fused-loss" "v1 --fused-loss" "v1 --lena-loss" "v5 --fused-loss" "v6 --fused-loss" "v4"; do
  for rev in 1 0; do
    DLADMM_BWD_REV=$rev timeout -k 10 120 python tools/bench_train.py --variant $spec \
      --steps 10 --warmup 2 > gpurun_out/t.json || exit 1
    python -c "import json,sys; r=json.load(open('gpurun_out/t.json')); r['bwd_rev_env']=$rev; print(json.dumps(r))" >> gpurun_out/r04_train2.jsonl
    python -c "import json; r=json.load(open('gpurun_out/t.json')); print('$spec rev=$rev', round(r['step_ms'],2), round(r['forward_ms'],2), round(r['backward_ms'],2))"
  done
done
