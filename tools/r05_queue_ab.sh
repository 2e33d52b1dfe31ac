#!/bin/bash
# Round 5: the bf16 forward as one persistent queue launch (dladmm_tile_bf16_queue.hip).  Its
# bit-identity tests first, then an interleaved A/B of the config-5 bench line (one-phase narrow,
# one-phase wide, queue with 1 / 2 / 4 lag classes), then a kernel trace of the queue mode.
#   tools/r05_queue_ab.sh -> gpurun_out/queue/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/queue
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread -k "queue" > $O/tests.log 2>&1 || { echo queue tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="--precision bf16 --m 1024 --n 4096 --batch 16384 --no-cpu-baseline"
for r in 1 2; do
for mode in "0 narrow 2" "0 wide 2" "1 wide 1" "1 wide 2" "1 wide 4"; do
set -- $mode
DLADMM_BF16_QUEUE=$1 DLADMM_BF16_TILE=$2 DLADMM_BF16_QUEUE_LAGS=$3 timeout -k 10 200 python bench.py $B --steps 10 --warmup 2 > $O/q$1_$2_$3.$r.json 2> $O/q$1_$2_$3.err || { echo "bench $mode failed"; tail -5 $O/q$1_$2_$3.err; exit 1; }
python -c "import json; d=json.loads(open('$O/q$1_$2_$3.$r.json').read().strip().splitlines()[-1]); print('queue=$1 tile=$2 lags=$3', round(d['ms_per_step'],3), 'ms', round(d['roofline']['kernel_ms'],3), 'kernel ms', round(d['roofline']['frac'],4))"
done
done
cd /tmp && export TMPDIR=/tmp
DLADMM_BF16_QUEUE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py $B --steps 3 --warmup 1 > $O/kt.log 2>&1 || exit 1
echo traces done
