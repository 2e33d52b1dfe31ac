#!/bin/bash
# Round 6 A/B (recorded in profiles/r06_rev_zlds_ab.json; the REV_ZLDS patch it measured --
# Z_k for BK2 staged by buffer LDS-DMA with counted waits -- lost and was reverted): the
# reverse / backward / training suites on the staged build, then one-process A/B timing against
# abl/zreg (register loads), fused-objective and per-layer-Z-cotangent forms.
mkdir -p gpurun_out/r06e
tools/gpu_run.sh \
  "900 python -u -m pytest tests/test_gpu_reverse.py tests/test_gpu_backward.py tests/test_gpu_training.py tests/test_gpu_lena.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06e/tests.log 2>&1" \
  "400 python -u tools/bench_bwd.py --reps 12 --libs main,d-ladmm_amd/lib/abl/zreg/libdladmm_hip.so > gpurun_out/r06e/ab_fused.json" \
  "400 python -u tools/bench_bwd.py --reps 12 --gz --libs main,d-ladmm_amd/lib/abl/zreg/libdladmm_hip.so > gpurun_out/r06e/ab_gz.json"
