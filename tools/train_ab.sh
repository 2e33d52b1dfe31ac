#!/bin/bash
# backward GPU tests + training-step bench and kernel stats (saved-P backward)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/train
timeout -k 10 400 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_training.py tests/test_gpu_smoke.py -x -q --timeout 120 --timeout-method thread > gpurun_out/train/tests.log 2>&1 || { tail -40 gpurun_out/train/tests.log; exit 1; }
tail -2 gpurun_out/train/tests.log
bash tools/train_prof.sh || exit 1
cat gpurun_out/train/fused.json gpurun_out/train/torchloss.json
