#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/r04l2
timeout -k 10 300 python -u -m pytest tests/test_gpu_lena.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04l2/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04l2/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/bench_lena.py > gpurun_out/r04l2/lena.json && cat gpurun_out/r04l2/lena.json || exit 1
timeout -k 10 200 python tools/bench_train.py --variant v1 --lena-fused --steps 10 --warmup 2 > gpurun_out/r04l2/train.json || exit 1
python -c "import json; r=json.load(open('gpurun_out/r04l2/train.json')); print(round(r['step_ms'],2), round(r['forward_ms'],2), round(r['backward_ms'],2))"
