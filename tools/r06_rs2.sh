#!/bin/bash
# Round 6: path 5 with V1, saved products and the fused objective (training forwards): its
# tests, the training suites that now run small batches on it, then where path 5 beats path 1
# as the batch grows (tools/bench_fwd_ab.py: threshold builds rs4 / rs8 = up to 4 / 8
# workgroups per CU; config 2 is B = 10,000).
mkdir -p gpurun_out/r06n
tools/gpu_run.sh \
  "300 python -u -m pytest tests/test_gpu_rowsplit.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06n/rs_tests.log 2>&1" \
  "900 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_training.py tests/test_gpu_lena.py tests/test_gpu_reverse.py tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06n/tests.log 2>&1" \
  "600 python -u tools/bench_fwd_ab.py --libs main,d-ladmm_amd/lib/abl/rs4/libdladmm_hip.so,d-ladmm_amd/lib/abl/rs8/libdladmm_hip.so --batches 4096,8192,10000,16384,32768 --reps 8 --no-rowsplit > gpurun_out/r06n/fwd_ab.json 2> gpurun_out/r06n/fwd_ab.err" \
  "300 python -u tools/bench_train.py --batch 25 --steps 50 --warmup 5 --fused-loss > gpurun_out/r06n/v4_b25_fused.json 2> gpurun_out/r06n/v4_b25_fused.err" \
  "300 python -u tools/bench_train.py --batch 25 --steps 50 --warmup 5 > gpurun_out/r06n/v4_b25.json 2> gpurun_out/r06n/v4_b25.err" \
  "300 python -u tools/bench_train.py --batch 20 --steps 50 --warmup 5 --variant v1 --lena-loss --lena-fused > gpurun_out/r06n/v1_b20_lena.json 2> gpurun_out/r06n/v1_b20_lena.err"
