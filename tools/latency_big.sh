#!/bin/bash
# tools/latency for 2 rank processes at 4 .. 64 MiB per rank: graph replay
# against the sliced interpreter with more and larger slices than the
# defaults.  JSON lines into gpurun_out/latency_big.jsonl.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run_pair() {  # label count env...
  local label=$1 count=$2; shift 2
  local d
  d=$(mktemp -d)
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 0 2 "file:$d" $count 300 >> gpurun_out/latency_big.jsonl &
  local p0=$!
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 1 2 "file:$d" $count 300 >> gpurun_out/latency_big.jsonl &
  local p1=$!
  wait $p0 || return 1
  wait $p1 || return 1
  rm -rf "$d"
}
for count in 1048576 4194304 16777216; do
  run_pair graph $count GLOO_AMD_GRAPH=1 || exit 1
  run_pair sliced_256x32k $count GLOO_AMD_INTERP_MAX_SLICES=256 || exit 1
  run_pair sliced_256x64k $count GLOO_AMD_INTERP_MAX_SLICES=256 GLOO_AMD_INTERP_SLICE_BYTES=65536 || exit 1
  run_pair sliced_128x128k $count GLOO_AMD_INTERP_MAX_SLICES=128 GLOO_AMD_INTERP_SLICE_BYTES=131072 || exit 1
done
cat gpurun_out/latency_big.jsonl
