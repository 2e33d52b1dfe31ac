#!/bin/bash
# Reverse sweep without the T_k loads (Var_{k+1} from the recomputed L_k, T_{k+1}): the reverse /
# backward / training / graph / lena tests, then fused-loss training steps (reverse path) per
# variant and the lena step.  Logs in gpurun_out/r04r3/.
set -o pipefail
O=gpurun_out/r04r3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_reverse.py tests/test_gpu_backward.py \
  tests/test_gpu_training.py tests/test_gpu_graph.py tests/test_gpu_lena.py -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
: > $O/train.jsonl
for spec in "v4 --fused-loss" "v1 --fused-loss" "v2 --fused-loss" "v3 --fused-loss" "v5 --fused-loss" "v6 --fused-loss" "v1 --lena-fused" "v4"; do
  timeout -k 10 120 python tools/bench_train.py --variant $spec --steps 10 --warmup 2 > $O/t.json || exit 1
  cat $O/t.json >> $O/train.jsonl
  python -c "import json; r=json.load(open('$O/t.json')); print('$spec', round(r['step_ms'],2), round(r['forward_ms'],2), round(r['backward_ms'],2))"
done
echo done
