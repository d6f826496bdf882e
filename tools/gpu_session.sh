#!/bin/bash
# Run a sequence of GPU steps on the gpurun box, each under its own time limit.
# Continue past an ordinary test failure (exit 1) but stop at anything that
# looks like a crash, abort, fault or timeout.  Usage:
#   tools/gpu_session.sh "<limit_s>:<name>:<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  limit="${spec%%:*}"; rest="${spec#*:}"; name="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${limit}s): $cmd" | tee -a gpurun_out/session.log
  timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc" | tee -a gpurun_out/session.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: step $name ended with $rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
