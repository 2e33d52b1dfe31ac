#!/bin/bash
# Training step with the reverse-sweep backward kernel vs the per-layer backward kernels
# (DLADMM_BWD_REV=0), interleaved on one box, then rocprofv3 kernel stats of the reverse form.
#   tools/rev_ab.sh  -> gpurun_out/rev/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/rev
for r in 1 2; do
  for mode in rev per; do
    if [ $mode = per ]; then export DLADMM_BWD_REV=0; else unset DLADMM_BWD_REV; fi
    timeout -k 10 200 python tools/bench_train.py --fused-loss > gpurun_out/rev/$mode.$r.json 2> gpurun_out/rev/$mode.err || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/rev/$mode.$r.json').read().strip().splitlines()[-1]); print('$mode', {k: d[k] for k in d if 'ms' in k or 'frac' in k})"
  done
done
unset DLADMM_BWD_REV
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rev/kt -o run -- python3 $R/tools/bench_train.py --fused-loss --steps 5 --warmup 1 > $R/gpurun_out/rev/kt.log 2>&1 || exit 1
