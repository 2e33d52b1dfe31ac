#!/bin/bash
# Round 5: config 5 (bf16 tiles) -- where a stage's LDS-DMA pieces issue in the main loop
# (DLADMM_TILE_DPOS ablation builds of tools/ablate.py --unit dladmm_tile_bf16.hip, same results):
# config-5 parity tests on each build, then the config-5 bench line, interleaved -> gpurun_out/tdpos/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/tdpos
mkdir -p $O
B="--precision bf16 --m 1024 --n 4096 --batch 16384 --no-cpu-baseline --no-cfg3 --no-split --no-train --steps 5 --warmup 2"
for v in ${VARIANTS:-tdpos1 tdpos2}; do
  L=$R/d-ladmm_amd/lib/abl/$v/libdladmm_hip.so
  DLADMM_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread > $O/$v.tests.log 2>&1 || { echo "$v tests failed"; tail -20 $O/$v.tests.log; exit 1; }
  echo "$v $(tail -1 $O/$v.tests.log)"
done
for r in 1 2 3; do
for v in main ${VARIANTS:-tdpos1 tdpos2}; do
  if [ $v = main ]; then L=""; else L=$R/d-ladmm_amd/lib/abl/$v/libdladmm_hip.so; fi
  DLADMM_LIB=$L timeout -k 10 200 python $R/bench.py $B > $O/$v.$r.json 2> $O/$v.err || { echo "$v failed"; tail -5 $O/$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/$v.$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', r.get('kernel_ms'), r.get('frac'), d['ms_per_step'])"
done
done
