#!/bin/bash
# Run GPU steps in order; stop at the first step that faults, aborts, segfaults or times out
# (exit >= 124 or killed by a signal).  Ordinary test failures (exit 1) do not stop later steps.
# usage: tools/gpu_run.sh "<seconds> <cmd...>" ["<seconds> <cmd...>" ...]   (logs in gpurun_out/)
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  i=$((i+1))
  secs=${spec%% *}
  cmd=${spec#* }
  echo "[gpu_run] step $i (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd"
  rc=$?
  echo "[gpu_run] step $i rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "[gpu_run] stopping: step $i ended with rc=$rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
