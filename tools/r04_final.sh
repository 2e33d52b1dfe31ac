#!/bin/bash
# Round-4 measurement set on one MI355X (logs and profiles under gpurun_out/r04f/):
#   1. the whole GPU test suite (parity log -> r04_parity.json)   2. smoke()
#   3. the default bench line                                      4. rocprofv3 kernel trace + stats
#   5. PMC passes: FETCH_SIZE, WRITE_SIZE, SQ (MFMA busy, clock)  (tools/profile.sh)
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/r04f
O=gpurun_out/r04f
timeout -k 10 700 env DLADMM_PARITY_JSON=$O/r04_parity.json python -u -m pytest tests -m gpu -q \
  --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?"; tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -5 $O/bench.err; exit 1; }
python -c "import json; r=json.load(open('$O/bench.json')); print('bench', r['value'], r['roofline']['frac'], r['roofline']['kernel_ms'])"
STEPS=20 bash tools/profile.sh || { echo profile failed; exit 1; }
cp -r gpurun_out/prof $O/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/train_prof -o run \
  -- python3 $R/tools/bench_train.py --fused-loss --steps 10 --warmup 2 > $R/$O/train_prof.log 2>&1 \
  || { echo train profile failed; exit 1; }
echo done
