#!/bin/bash
# Round 6: path 6 final form (unrolled exchange loads, the next pass's fragments fetched behind
# them): smoke, the suites it serves, forward A/B against paths 5 / 1, the f2/f3 lines, the
# reference loops' training steps.
mkdir -p gpurun_out/r06w
tools/gpu_run.sh \
  "120 python -u tools/xs_smoke.py > gpurun_out/r06w/smoke.txt 2>&1" \
  "900 python -u -m pytest tests/test_gpu_rowsplit.py tests/test_capi.py tests/test_gpu_training.py tests/test_gpu_lena.py tests/test_gpu_lskm.py tests/test_gpu_eval.py tests/test_gpu_configs.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06w/tests.log 2>&1" \
  "300 python -u tools/bench_fwd_ab.py --batches 20,100,256,512,1000 --flag-set 0,128,64 --reps 10 > gpurun_out/r06w/fwd_ab.json 2> gpurun_out/r06w/fwd_ab.err" \
  "300 python -u tools/bench_eval.py --ab > gpurun_out/r06w/eval.json 2> gpurun_out/r06w/eval.err" \
  "300 python -u tools/bench_train.py --batch 20 --steps 50 --warmup 5 --variant v1 --lena-loss --lena-fused > gpurun_out/r06w/v1_b20_lena.json 2> gpurun_out/r06w/v1_b20_lena.err" \
  "300 python -u tools/bench_train.py --batch 25 --steps 50 --warmup 5 --fused-loss > gpurun_out/r06w/v4_b25_fused.json 2> gpurun_out/r06w/v4_b25_fused.err"
