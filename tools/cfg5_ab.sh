#!/bin/bash
# Config-5 bf16 tile forms: the bf16 GPU tests, then an interleaved A/B of the bench line
#   TILES="narrow ws" tools/cfg5_ab.sh    -> gpurun_out/cfg5/
set -u
mkdir -p gpurun_out/cfg5
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cfg5/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/cfg5/tests.log; exit 1; }
tail -2 gpurun_out/cfg5/tests.log
for r in 1 2; do
for t in ${TILES:-narrow ws}; do
DLADMM_BF16_TILE=$t timeout -k 10 200 python bench.py --precision bf16 --m 1024 --n 4096 --batch 16384 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/cfg5/$t.$r.json 2> gpurun_out/cfg5/$t.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/cfg5/$t.$r.json').read().strip().splitlines()[-1]); print('$t', round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,3), 'M/s', round(d['roofline']['frac'],4))"
done
done
