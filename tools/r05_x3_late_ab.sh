#!/bin/bash
# Round 5: split-f16 forward, ring DMA group issued after the barrier step's MFMAs (X3_DMA_LATE
# ablation build of tools/ablate.py --unit dladmm_fused_x3.hip) against the shipped placement:
# split parity tests on the build, then the bench's split_f16 sub-line, interleaved
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/x3late
mkdir -p $O
V=${VARIANTS:-x3late}
for v in $V; do
  DLADMM_LIB=$R/d-ladmm_amd/lib/abl/$v/libdladmm_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread -k "not weight_gradient and not bit_identical" > $O/$v.tests.log 2>&1 || { echo "$v tests failed"; tail -20 $O/$v.tests.log; exit 1; }
  echo "$v $(tail -1 $O/$v.tests.log)"
done
B="--no-cpu-baseline --no-cfg3 --no-train --steps 20 --warmup 5"
for r in 1 2 3; do
for v in main $V; do
  if [ $v = main ]; then L=""; else L=$R/d-ladmm_amd/lib/abl/$v/libdladmm_hip.so; fi
  DLADMM_LIB=$L timeout -k 10 200 python $R/bench.py $B > $O/$v.$r.json 2> $O/$v.err || { echo "$v failed"; tail -5 $O/$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/$v.$r.json').read().strip().splitlines()[-1]); x=d['split_f16']; print('$v', round(x['kernel_ms'],4), 'split kernel ms', round(x['value']/1e6,3), 'M samples/s')"
done
done
