#!/bin/bash
# Round 5: where the pipelined bf16 G1 kernel's time goes.  Kernel traces of config 5 with the
# regular library and the ablation builds of tools/ablate.py --unit dladmm_tile_bf16_pipe.hip
# (pnoepi: no epilogue, pnomfma: no MFMA, pskel: neither) -> gpurun_out/pabl/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pabl
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="--precision bf16 --m 1024 --n 4096 --batch 16384 --no-cpu-baseline --steps 3 --warmup 1"
for v in ${VARIANTS:-full pnoepi pnomfma pskel}; do
  if [ $v = full ]; then L=""; else L=$R/d-ladmm_amd/lib/abl/$v/libdladmm_hip.so; fi
  DLADMM_BF16_PIPE=1 DLADMM_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- python3 $R/bench.py $B > $O/$v.log 2>&1 || exit 1
  python3 - $O/$v $v <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "tile" in r["Kernel_Name"]:
            d[r["Kernel_Name"].split("(")[0][-40:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
for k, v in sorted(d.items()):
    print(sys.argv[2], k, len(v), round(sum(v) / len(v), 1), "us")
PY
done
