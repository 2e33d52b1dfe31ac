#!/bin/bash
# fused main_lena objective: GPU tests, then V1 training steps (torch-op lena loss vs fused)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04l
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_lena.py -x -v -s --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_train.py --variant v1 --lena-fused --steps 10 --warmup 2 > $O/train_fused.json 2> $O/train_fused.err || { tail -5 $O/train_fused.err; exit 1; }
tail -1 $O/train_fused.json | cut -c1-600
timeout -k 10 200 python tools/bench_train.py --variant v1 --lena-loss --steps 10 --warmup 2 > $O/train_torch.json 2> $O/train_torch.err || { tail -5 $O/train_torch.err; exit 1; }
tail -1 $O/train_torch.json | cut -c1-600
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python3 $R/tools/bench_train.py --variant v1 --lena-fused --steps 5 --warmup 1 > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
echo done
