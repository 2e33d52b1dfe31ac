#!/bin/bash
# Round 5: bf16 G1 on the persistent pipelined kernel (dladmm_tile_bf16_pipe.hip).  The pipe
# bit-identity tests first, then an interleaved A/B of the config-5 bench line, then a kernel
# trace of each mode.   tools/r05_pipe_ab.sh -> gpurun_out/pipe/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pipe
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread -k "pipelined" > $O/tests.log 2>&1 || { echo pipe tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="--precision bf16 --m 1024 --n 4096 --batch 16384 --no-cpu-baseline"
for r in 1 2; do
for mode in 0 1; do
DLADMM_BF16_PIPE=$mode timeout -k 10 200 python bench.py $B --steps 10 --warmup 2 > $O/p$mode.$r.json 2> $O/p$mode.err || exit 1
python -c "import json; d=json.loads(open('$O/p$mode.$r.json').read().strip().splitlines()[-1]); print('pipe=$mode', round(d['ms_per_step'],3), 'ms', round(d['roofline']['kernel_ms'],3), 'kernel ms', round(d['roofline']['frac'],4))"
done
done
cd /tmp && export TMPDIR=/tmp
for mode in 0 1; do
DLADMM_BF16_PIPE=$mode timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$mode -o run -- python3 $R/bench.py $B --steps 3 --warmup 1 > $O/kt$mode.log 2>&1 || exit 1
done
echo traces done
