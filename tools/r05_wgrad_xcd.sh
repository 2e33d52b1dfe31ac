#!/bin/bash
# Round 5: split-f16 weight gradient, XCD-grouped tiles (DLADMM_WGRAD_X3_XCD=1, default: the
# tiles of one chunk and layer on one XCD, so its L2 serves the shared V rows) against
# consecutive workgroup ids (=0): tests, then f32_split training-step kernel traces of both ->
# gpurun_out/wxcd/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/wxcd
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread -k "weight_gradient or training_saves" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
for xv in 1 0; do
  DLADMM_WGRAD_X3_XCD=$xv timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x$xv$i -o run -- python3 $R/tools/bench_train.py --variant v4 --fused-loss --precision f32_split > $O/x$xv$i.log 2>&1 || exit 1
  python3 - $O/x$xv$i $xv <<'PY'
import csv, glob, sys, json
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wgrad_x3" in r["Name"]:
            print("XCD", sys.argv[2], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
  grep -o '"step_ms": [0-9.]*' $O/x$xv$i.log | tail -1
done
done
