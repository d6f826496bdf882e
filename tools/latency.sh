#!/bin/bash
# tools/latency for 2 rank processes: HD allreduce of 1 KiB .. 1 MiB under
# each launch mode (executor.h): the one-launch interpreter (default for
# small plans), hipGraph replay, step-by-step enqueue.  JSON lines into
# gpurun_out/latency.jsonl.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run_pair() {  # label count env...
  local label=$1 count=$2; shift 2
  local d
  d=$(mktemp -d)
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 0 2 "file:$d" $count 1000 >> gpurun_out/latency.jsonl &
  local p0=$!
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 1 2 "file:$d" $count 1000 >> gpurun_out/latency.jsonl &
  local p1=$!
  wait $p0 || return 1
  wait $p1 || return 1
  rm -rf "$d"
}
for count in 256 4096 16384 262144; do
  run_pair interp $count GLOO_AMD_INTERP_BYTES=1048576 || exit 1
  run_pair graph $count GLOO_AMD_GRAPH=1 || exit 1
  run_pair eager $count GLOO_AMD_GRAPH=0 GLOO_AMD_INTERP=0 || exit 1
done
cat gpurun_out/latency.jsonl
