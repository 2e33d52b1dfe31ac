#!/bin/bash
# One rocprofv3 PMC pass (+ kernel trace) over a short bench run.
#   tools/pmc.sh <name> <counter> [<counter> ...]     -> gpurun_out/prof/<name>/
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
name=$1; shift
mkdir -p $R/gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $R/gpurun_out/prof/$name -o run \
  -- python3 $R/bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $R/gpurun_out/prof/$name.log 2>&1
