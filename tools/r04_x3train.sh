#!/bin/bash
# split-f16 training: split / backward / reverse / training / graph / lena tests, then training
# steps on both precisions
set -o pipefail
O=gpurun_out/r04x3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_backward.py \
  tests/test_gpu_reverse.py tests/test_gpu_training.py tests/test_gpu_graph.py tests/test_gpu_lena.py \
  -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in v4 v6; do
  for prec in f32 f32_split; do
    timeout -k 10 120 python tools/bench_train.py --variant $v --fused-loss --precision $prec --steps 10 --warmup 2 > $O/t.json || exit 1
    python -c "import json; r=json.load(open('$O/t.json')); print('$v $prec', round(r['step_ms'],2), round(r['forward_ms'],2), round(r['backward_ms'],2))"
    cat $O/t.json >> $O/train.jsonl
  done
done
echo done
