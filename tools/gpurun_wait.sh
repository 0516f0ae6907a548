#!/bin/bash
# Submit one gpurun call, re-submitting only while the pool reports no free slot or box
# (exit 3 / "status=transient": nothing ran, nothing was charged).  Never re-runs a command
# that started on a GPU.   usage: tools/gpurun_wait.sh <outfile> <timeout> <command>
out=$1; to=$2; shift 2
for k in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$out"; then sleep 60; continue; fi
  exit $rc
done
exit 3
