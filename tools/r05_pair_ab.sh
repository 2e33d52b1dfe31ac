#!/bin/bash
# Round 5: bf16 paired-halves launches (dladmm_tile_bf16_pair.hip).  The bf16 GPU tests (incl. the
# paired-vs-one-phase bit-identity test), then an interleaved A/B of the config-5 bench line:
#   DLADMM_BF16_PAIR=0 (one phase per launch) vs paired with F = 1000 / 500 permille
#   tools/r05_pair_ab.sh   -> gpurun_out/pair/
set -u
mkdir -p gpurun_out/pair
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pair/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/pair/tests.log; exit 1; }
tail -2 gpurun_out/pair/tests.log
for r in 1 2; do
for cfg in "0 1000" "1 1000" "1 500"; do
set -- $cfg
DLADMM_BF16_PAIR=$1 DLADMM_BF16_PAIR_F=$2 timeout -k 10 200 python bench.py --precision bf16 --m 1024 --n 4096 --batch 16384 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/pair/p$1_$2.$r.json 2> gpurun_out/pair/p$1_$2.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/pair/p$1_$2.$r.json').read().strip().splitlines()[-1]); print('pair=$1 F=$2', round(d['ms_per_step'],3), 'ms', round(d['roofline']['kernel_ms'],3), 'kernel ms', round(d['value']/1e6,3), 'M/s', round(d['roofline']['frac'],4))"
done
done
