#!/bin/bash
# Round 5: split-f16 weight gradient (dladmm_wgrad_x3.hip) -- its tests, then the f32_split
# training step with it and without it (DLADMM_WGRAD_X3=0), interleaved, and a kernel trace.
#   tools/r05_wgrad_x3.sh -> gpurun_out/wx3/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/wx3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread -k "weight_gradient or training_saves" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
for x in 0 1; do
DLADMM_WGRAD_X3=$x timeout -k 10 200 python tools/bench_train.py --variant v4 --fused-loss --precision f32_split > $O/t$x.$r.json 2> $O/t$x.err || { echo "bench failed"; tail -5 $O/t$x.err; exit 1; }
python -c "import json; d=json.loads(open('$O/t$x.$r.json').read().strip().splitlines()[-1]); print('x3=$x', round(d['step_ms'],3), 'step ms', round(d['backward_ms'],3), 'bwd ms')"
done
done
cd /tmp && export TMPDIR=/tmp
DLADMM_WGRAD_X3=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/tools/bench_train.py --variant v4 --fused-loss --precision f32_split > $O/kt.log 2>&1 || exit 1
echo traces done
