#!/bin/bash
# Round 6, measurement call: (1) the saved-product forward in isolation vs inference
# (tools/savep_ab.py), (2) the clock the training step's kernels hold (GRBM_GUI_ACTIVE per
# dispatch, tools/bench_train.py V4 fused loss) beside the inference headline's, (3) the
# training-step kernel breakdowns (V1, V4 fp32, V4 split-f16), (4) the headline kernel's
# rocprofv3 summary and HBM traffic passes (FETCH_SIZE, WRITE_SIZE: separate passes), (5) the
# N = 2 launcher on gloo (two ranks on the one card: control path only).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r06m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
st() { echo "[r06_run5] $*"; }
st savep_ab
timeout -k 10 300 python3 $R/tools/savep_ab.py > $O/savep_ab.json 2> $O/savep_ab.err || exit 1
st train_clock
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  --output-format csv -d $O/train_clock -o run -- python3 $R/tools/bench_train.py --variant v4 \
  --fused-loss --steps 5 --warmup 2 > $O/train_clock.log 2>&1 || exit 1
st head_clock
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  --output-format csv -d $O/head_clock -o run -- python3 $R/bench.py --no-cfg3 --no-train \
  --no-cpu-baseline --no-split --steps 5 --warmup 1 > $O/head_clock.log 2>&1 || exit 1
for v in v1 v4; do
  st train_$v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train_$v -o run \
    -- python3 $R/tools/bench_train.py --variant $v --fused-loss --steps 10 --warmup 2 \
    > $O/train_$v.log 2>&1 || exit 1
done
st train_v4_split
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train_v4s -o run \
  -- python3 $R/tools/bench_train.py --variant v4 --fused-loss --precision f32_split --steps 10 \
  --warmup 2 > $O/train_v4s.log 2>&1 || exit 1
st head_stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/head_stats -o run \
  -- python3 $R/bench.py --no-cfg3 --no-train --no-cpu-baseline --no-split --steps 20 \
  --warmup 3 > $O/head_stats.json 2> $O/head_stats.err || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  st head_$c
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/head_$c -o run \
    -- python3 $R/bench.py --no-cfg3 --no-train --no-cpu-baseline --no-split --steps 3 \
    --warmup 1 > $O/head_$c.log 2>&1 || exit 1
done
st launcher_gloo2
cd $R
DLADMM_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --no-cfg3 --no-train \
  --no-cpu-baseline --steps 5 --warmup 1 > $O/launcher_gloo2.json 2> $O/launcher_gloo2.err || exit 1
st done
