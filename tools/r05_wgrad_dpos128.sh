#!/bin/bash
# Round 5: split-f16 weight gradient at m = 64, n = 256 (128-row V tiles, two workgroups per CU): LDS-DMA
# after the MFMAs (DLADMM_WGRAD_X3_DPOS=1) against right after the fragment reads (=0)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/w128
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
for v in 1 0; do
  DLADMM_WGRAD_X3_DPOS=$v timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r$v$i -o run -- python3 $R/tools/bench_train.py --variant v4 --fused-loss --precision f32_split --m 64 --n 256 > $O/r$v$i.log 2>&1 || exit 1
  python3 - $O/r$v$i $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wgrad_x3" in r["Name"]:
            print("DPOS", sys.argv[2], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
done
