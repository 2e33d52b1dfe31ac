#!/bin/bash
# Lena objective tests (incl. the retained-graph double backward).  Log: gpurun_out/r04l3/tests.log
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/r04l3
timeout -k 10 300 python -u -m pytest tests/test_gpu_lena.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04l3/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04l3/tests.log; exit $rc
