#!/bin/bash
# Round 6: the row-split reverse sweep (dladmm_bwd_path 2) -- its tests, the backward / training
# suites that now run small batches on it, the small-batch training steps, backward timing.
mkdir -p gpurun_out/r06q
tools/gpu_run.sh \
  "400 python -u -m pytest tests/test_gpu_rowsplit.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06q/rs_tests.log 2>&1" \
  "900 python -u -m pytest tests/test_gpu_reverse.py tests/test_gpu_backward.py tests/test_gpu_training.py tests/test_gpu_lena.py tests/test_gpu_graph.py tests/test_gpu_split.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06q/tests.log 2>&1" \
  "300 python -u tools/bench_train.py --batch 25 --steps 50 --warmup 5 --fused-loss > gpurun_out/r06q/v4_b25_fused.json 2> gpurun_out/r06q/v4_b25_fused.err" \
  "300 python -u tools/bench_train.py --batch 25 --steps 50 --warmup 5 > gpurun_out/r06q/v4_b25.json 2> gpurun_out/r06q/v4_b25.err" \
  "300 python -u tools/bench_train.py --batch 20 --steps 50 --warmup 5 --variant v1 --lena-loss --lena-fused > gpurun_out/r06q/v1_b20_lena.json 2> gpurun_out/r06q/v1_b20_lena.err" \
  "200 python -u tools/bench_bwd.py --reps 20 --batch 25 > gpurun_out/r06q/bwd25.json" \
  "200 python -u tools/bench_bwd.py --reps 20 --batch 4096 > gpurun_out/r06q/bwd4096.json" \
  "200 python -u tools/bench_bwd.py --reps 20 --batch 10000 > gpurun_out/r06q/bwd10000.json" \
  "200 python -u tools/bench_bwd.py --reps 20 --batch 25 --no-rowsplit > gpurun_out/r06q/bwd25_p1.json" \
  "200 python -u tools/bench_bwd.py --reps 20 --batch 4096 --no-rowsplit > gpurun_out/r06q/bwd4096_p1.json" \
  "200 python -u tools/bench_bwd.py --reps 20 --batch 10000 --no-rowsplit > gpurun_out/r06q/bwd10000_p1.json"
