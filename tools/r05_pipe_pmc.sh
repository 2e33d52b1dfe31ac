#!/bin/bash
# Round 5: counters of config 5's G1 kernels -- the one-phase tile kernel, the pipelined G1
# kernel, and the pipelined kernel with its Z_k / packed stores sent to null views (ablation build
# pnost of tools/ablate.py --unit dladmm_tile_bf16_pipe.hip) -> gpurun_out/pipepmc/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pipepmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="--precision bf16 --m 1024 --n 4096 --batch 16384 --no-cpu-baseline --steps 3 --warmup 1"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_BARRIER SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum"
P3="TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
for mode in onephase pipe pnost; do
  case $mode in
    onephase) export DLADMM_BF16_PIPE=0 DLADMM_LIB= ;;
    pipe) export DLADMM_BF16_PIPE=1 DLADMM_LIB= ;;
    pnost) export DLADMM_BF16_PIPE=1 DLADMM_LIB=$R/d-ladmm_amd/lib/abl/pnost/libdladmm_hip.so ;;
  esac
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $O/${mode}_p$i -o run \
      -- python3 $R/bench.py $B > $O/${mode}_p$i.log 2>&1 || exit 1
  done
done
echo pmc done
