#!/bin/bash
# Round 5: is the split-f16 weight gradient bound by its strided operand reads?  The f32_split
# training step with the regular build against the probe build wblk (tools/ablate.py --unit
# dladmm_wgrad_x3.hip -DWX3_EXP=1: G / V read as if column-blocked, contiguous 16-KiB tiles;
# wrong gradients), kernel traces -> gpurun_out/wblk/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/wblk
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-main wblk}; do
  if [ $v = main ]; then L=""; else L=$R/d-ladmm_amd/lib/abl/$v/libdladmm_hip.so; fi
  DLADMM_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/tools/bench_train.py --variant v4 --fused-loss --precision f32_split > $O/$v.log 2>&1 || exit 1
  python3 - $O/$v $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wgrad" in r["Name"]:
            print(sys.argv[2], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
