#!/bin/bash
# Kernel timeline of tools/latency (LAT_P rank processes, default 2, HD fp32
# sum) at the given element counts: rank 0 under rocprofv3 --kernel-trace
# (full trace, CSV), the others plain.  Env passes through (GLOO_AMD_GRAPH=1 ...).
#   tools/latency_trace.sh LABEL COUNT...   -> gpurun_out/trace_<LABEL>_<COUNT>/
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${LAT_P:-2}
label=$1; shift
for count in "$@"; do
  d=$(mktemp -d)
  timeout -k 5 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_${label}_${count} -o lat \
    -- ./tools/latency 0 $P "file:$d" $count 300 > gpurun_out/trace_${label}_${count}.json &
  pids=($!)
  for r in $(seq 1 $((P - 1))); do
    timeout -k 5 120 ./tools/latency $r $P "file:$d" $count 300 > /dev/null &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait $p || exit 1; done
  rm -rf "$d"
  cat gpurun_out/trace_${label}_${count}.json
done
