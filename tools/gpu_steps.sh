#!/bin/bash
# Run GPU steps in sequence on the gpurun box. Each step: `name seconds command...`.
# An ordinary failure (pytest rc 1/2) moves on; a timeout, abort or crash (rc >= 124, 134, 139)
# ends the script so nothing else touches a possibly wedged GPU.
mkdir -p gpurun_out
: > gpurun_out/summary.txt
while [ $# -gt 0 ]; do
  spec="$1"; shift
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "== $name ($secs s): $cmd" >> gpurun_out/summary.txt
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc" >> gpurun_out/summary.txt
  tail -3 "gpurun_out/$name.log" >> gpurun_out/summary.txt
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fatal rc=$rc in $name: stopping" >> gpurun_out/summary.txt
    cat gpurun_out/summary.txt
    exit $rc
  fi
done
cat gpurun_out/summary.txt
