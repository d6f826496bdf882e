#!/bin/bash
# tools/latency for 2 rank processes: HD allreduce of 1 KiB .. 16 MiB under
# each launch mode (executor.h): the defaults (sliced interpreter up to
# 32 x 64 KiB messages, graph replay above), the interpreter held to one
# workgroup, hipGraph replay, step-by-step enqueue.  JSON lines into
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
for count in 256 16384 65536 262144 1048576 4194304; do
  run_pair default $count || exit 1
  run_pair one_workgroup $count GLOO_AMD_INTERP_SLICE_BYTES=1000000000 || exit 1
  run_pair graph $count GLOO_AMD_GRAPH=1 || exit 1
  run_pair eager $count GLOO_AMD_GRAPH=0 GLOO_AMD_INTERP=0 || exit 1
done
cat gpurun_out/latency.jsonl
