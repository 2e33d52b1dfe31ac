#!/bin/bash
# config-2 row-split skeleton (tools/probe/cfg2_split2.hip): timings, then one counter pass
# (L1 -> L2 read requests and latency, clock) -> gpurun_out/r04c2/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04c2
mkdir -p $O
timeout -k 10 120 $R/tools/probe/cfg2_split2 > $O/probe.json 2> $O/probe.err || { echo probe failed; exit 1; }
cat $O/probe.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY GRBM_GUI_ACTIVE \
  --output-format csv -d $O/pmc -o run -- $R/tools/probe/cfg2_split2 > $O/pmc.log 2>&1 || { echo pmc failed; exit 1; }
echo done
