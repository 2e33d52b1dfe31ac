#!/bin/bash
# Round 5: why paired-halves bf16 launches are slower.  Timing A/B over the dispatch-order knob,
# then per mode one PMC pass with L2 hits / misses + MFMA busy and one with FETCH_SIZE.
#   tools/r05_pair_pmc.sh -> gpurun_out/pairpmc/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pairpmc
mkdir -p $O
B="--precision bf16 --m 1024 --n 4096 --batch 16384 --no-cpu-baseline"
for r in 1 2; do
for cfg in "0 1000" "1 1" "1 250"; do
set -- $cfg
DLADMM_BF16_PAIR=$1 DLADMM_BF16_PAIR_F=$2 timeout -k 10 200 python $R/bench.py $B --steps 10 --warmup 2 > $O/p$1_$2.$r.json 2> $O/p$1_$2.err || exit 1
python -c "import json; d=json.loads(open('$O/p$1_$2.$r.json').read().strip().splitlines()[-1]); print('pair=$1 F=$2', round(d['ms_per_step'],3), 'ms', round(d['roofline']['kernel_ms'],3), 'kernel ms')"
done
done
cd /tmp && export TMPDIR=/tmp
for cfg in "0 1000" "1 1"; do
set -- $cfg
export DLADMM_BF16_PAIR=$1 DLADMM_BF16_PAIR_F=$2
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_a_$1 -o run \
  -- python3 $R/bench.py $B --steps 3 --warmup 1 > $O/pmc_a_$1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_b_$1 -o run \
  -- python3 $R/bench.py $B --steps 3 --warmup 1 > $O/pmc_b_$1.log 2>&1 || exit 1
done
echo pmc done
