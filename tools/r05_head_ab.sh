#!/bin/bash
# Round 5: headline fused-kernel A/B (bench line alone, interleaved): the regular library against
# the ablation builds named in VARIANTS (tools/ablate.py --unit dladmm_fused.hip)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/headab
mkdir -p $O
B="--no-cpu-baseline --no-cfg3 --no-split --no-train --steps 20 --warmup 5"
for r in 1 2 3; do
for v in main ${VARIANTS}; do
  if [ $v = main ]; then L=""; else L=$R/d-ladmm_amd/lib/abl/$v/libdladmm_hip.so; fi
  DLADMM_LIB=$L timeout -k 10 200 python $R/bench.py $B > $O/$v.$r.json 2> $O/$v.err || { echo "$v failed"; tail -5 $O/$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/$v.$r.json').read().strip().splitlines()[-1]); print('$v', round(d['roofline']['kernel_ms'],4), 'kernel ms', round(d['roofline']['frac'],4))"
done
done
