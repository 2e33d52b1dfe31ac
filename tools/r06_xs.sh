#!/bin/bash
# Round 6: path 6, the four-workgroup row split (dladmm_fused_xs.hip): a quick bit-equality /
# wall-time check, the row-split tests (both flavours), forward A/B at small batches, the f2/f3
# lines and the reference loops' training steps.
mkdir -p gpurun_out/r06x
tools/gpu_run.sh \
  "120 python -u tools/xs_smoke.py > gpurun_out/r06x/smoke.txt 2>&1" \
  "600 python -u -m pytest tests/test_gpu_rowsplit.py tests/test_capi.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06x/tests.log 2>&1" \
  "300 python -u tools/bench_fwd_ab.py --batches 20,100,256,512,1000 --flag-set 0,128,64 --reps 10 > gpurun_out/r06x/fwd_ab.json 2> gpurun_out/r06x/fwd_ab.err" \
  "300 python -u tools/bench_eval.py --ab > gpurun_out/r06x/eval.json 2> gpurun_out/r06x/eval.err" \
  "300 python -u tools/bench_train.py --batch 20 --steps 50 --warmup 5 --variant v1 --lena-loss --lena-fused > gpurun_out/r06x/v1_b20_lena.json 2> gpurun_out/r06x/v1_b20_lena.err"
