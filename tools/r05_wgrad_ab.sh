#!/bin/bash
# Round 5: split-f16 weight-gradient A/B on one environment switch.  Usage:
#   tools/r05_wgrad_ab.sh VAR "VAL1 VAL2" TAG [PRECISION [KERNEL]]
# runs the split tests, then training-step kernel traces (precision f32_split by default) with
# VAR=VAL1, VAR=VAL2 (twice, alternating) -> gpurun_out/TAG/ (the average per launch of kernels
# whose name contains KERNEL, default wgrad_x3, and the step time per run)
set -u
VAR=$1; VALS=$2; TAG=$3; PREC=${4:-f32_split}; KN=${5:-wgrad_x3}
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_reverse.py tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
for v in $VALS; do
  env $VAR=$v timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r$v$i -o run -- python3 $R/tools/bench_train.py --variant v4 --fused-loss --precision $PREC > $O/r$v$i.log 2>&1 || exit 1
  python3 - $O/r$v$i "$VAR=$v" $KN <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sys.argv[3] in r["Name"] and "reduce" not in r["Name"]:
            print(sys.argv[2], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
  grep -o '"step_ms": [0-9.]*' $O/r$v$i.log | tail -1
done
done
