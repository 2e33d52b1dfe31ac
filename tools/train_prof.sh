#!/bin/bash
# training-step bench (fused loss and torch-op loss) + rocprofv3 kernel stats of the fused-loss step
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/train
cd $R
timeout -k 10 200 python tools/bench_train.py --fused-loss > gpurun_out/train/fused.json 2> gpurun_out/train/fused.err || exit 1
timeout -k 10 200 python tools/bench_train.py > gpurun_out/train/torchloss.json 2> gpurun_out/train/torchloss.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/train/kt -o run -- python3 $R/tools/bench_train.py --fused-loss --steps 5 --warmup 1 > $R/gpurun_out/train/kt.log 2>&1 || exit 1
