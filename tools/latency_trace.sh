#!/bin/bash
# Kernel timeline of tools/latency (2 rank processes, HD fp32 sum) at the
# given element counts: rank 0 under rocprofv3 --kernel-trace (full trace,
# CSV), rank 1 plain.  Env passes through (GLOO_AMD_GRAPH=1 ...).
#   tools/latency_trace.sh LABEL COUNT...   -> gpurun_out/trace_<LABEL>_<COUNT>/
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
label=$1; shift
for count in "$@"; do
  d=$(mktemp -d)
  timeout -k 5 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_${label}_${count} -o lat \
    -- ./tools/latency 0 2 "file:$d" $count 300 > gpurun_out/trace_${label}_${count}.json &
  p0=$!
  timeout -k 5 120 ./tools/latency 1 2 "file:$d" $count 300 > /dev/null &
  p1=$!
  wait $p0 || exit 1
  wait $p1 || exit 1
  rm -rf "$d"
  cat gpurun_out/trace_${label}_${count}.json
done
