#!/bin/bash
# client-side wait for a free GPU slot: re-submit ONLY when gpurun reports that no box/slot was
# available or that access is backing off (nothing ran, nothing charged); any other outcome
# ends the loop
out=$1; shift
for i in $(seq 1 40); do
  timeout 2700 /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient" $out && grep -q "nothing was charged\|no free box right now\|backing off" $out; then
    sleep 90; continue
  fi
  echo "gpurun rc=$rc after $i tries" >> $out
  exit $rc
done
