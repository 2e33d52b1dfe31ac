#!/bin/bash
# Round 5: split-f16 weight-gradient A/B against ablation builds of tools/ablate.py --unit
# dladmm_wgrad_x3.hip (VARIANTS): split tests on each build, then alternating training-step
# kernel traces -> gpurun_out/wlib/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/wlib
mkdir -p $O
for v in ${VARIANTS}; do
  DLADMM_LIB=$R/d-ladmm_amd/lib/abl/$v/libdladmm_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread -k "weight_gradient or bit_identical" > $O/$v.tests.log 2>&1 || { echo "$v tests failed"; tail -20 $O/$v.tests.log; exit 1; }
  echo "$v $(tail -1 $O/$v.tests.log)"
done
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
for v in main ${VARIANTS}; do
  if [ $v = main ]; then L=""; else L=$R/d-ladmm_amd/lib/abl/$v/libdladmm_hip.so; fi
  DLADMM_LIB=$L timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v$i -o run -- python3 $R/tools/bench_train.py --variant v4 --fused-loss --precision f32_split > $O/$v$i.log 2>&1 || exit 1
  python3 - $O/$v$i $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wgrad_x3" in r["Name"]:
            print(sys.argv[2], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
done
