#!/bin/bash
# tools/latency for 2 rank processes at the mid sizes (HD
# 4 MiB and 16 MiB per rank) under launch-mode / copy-engine variants.
# JSON lines into gpurun_out/latency_mid.jsonl.
#   tools/latency_mid.sh [COUNT ...]
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run_pair() {  # label count env...
  local label=$1 count=$2; shift 2
  local d
  d=$(mktemp -d)
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 0 2 "file:$d" $count 400 >> gpurun_out/latency_mid.jsonl &
  local p0=$!
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 1 2 "file:$d" $count 400 > /dev/null &
  local p1=$!
  wait $p0 || return 1
  wait $p1 || return 1
  rm -rf "$d"
}
counts=${*:-"1048576 4194304"}
for count in $counts; do
  run_pair default $count || exit 1
  run_pair ref_route $count GLOO_AMD_MESH=0 || exit 1
  run_pair copy_kernel64 $count GLOO_AMD_COPY=kernel || exit 1
  run_pair copy_kernel256 $count GLOO_AMD_COPY=kernel GLOO_AMD_COPY_BLOCKS=256 || exit 1
  run_pair sliced64x64k $count GLOO_AMD_INTERP_MAX_SLICES=64 GLOO_AMD_INTERP_SLICE_BYTES=65536 || exit 1
  run_pair sliced128x32k $count GLOO_AMD_INTERP_MAX_SLICES=128 GLOO_AMD_INTERP_SLICE_BYTES=32768 || exit 1
  run_pair sliced128x128k $count GLOO_AMD_INTERP_MAX_SLICES=128 GLOO_AMD_INTERP_SLICE_BYTES=131072 || exit 1
  tail -7 gpurun_out/latency_mid.jsonl
done
