#!/bin/bash
# Developer helper: run one gpurun call, retrying ONLY when no box was ever
# prepared (status=transient / no box free: nothing ran, nothing charged).
# A call that ran is never retried.  Earlier results under gpurun_out/ are kept
# (round 6 lost two records to a clean-up here).  Usage: tools/gpurun_retry.sh <limit_s> '<command>'
t=$1; shift
cd "$(dirname "$0")/.." || exit 1
for i in 1 2 3 4 5; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > gpurun_last.log 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { grep -q "status=transient" gpurun_last.log && grep -q "run 0.0s" gpurun_last.log; }; then
    echo "no box (rc $rc), retry $i in 60 s"; sleep 60; continue
  fi
  break
done
tail -5 gpurun_last.log
exit $rc
