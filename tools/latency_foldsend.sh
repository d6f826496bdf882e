#!/bin/bash
# tools/latency for 2 rank processes, HD fp32 sum at the given counts, with
# the fold + forward fusion on (default), on with a release per workgroup
# (GLOO_AMD_FWD_RELEASE=each), off (GLOO_AMD_FOLD_SEND=0), and with every
# SEND on the copy kernel (256 workgroups),
# alternated REPS times.  JSON lines into gpurun_out/latency_foldsend.jsonl.
#   tools/latency_foldsend.sh REPS COUNT...
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run_pair() {  # label count env...
  local label=$1 count=$2; shift 2
  local d
  d=$(mktemp -d)
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 0 2 "file:$d" $count 400 >> gpurun_out/latency_foldsend.jsonl &
  local p0=$!
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 1 2 "file:$d" $count 400 > /dev/null &
  local p1=$!
  wait $p0 || return 1
  wait $p1 || return 1
  rm -rf "$d"
}
reps=$1; shift
for count in "$@"; do
  for rep in $(seq "$reps"); do
    run_pair fold_send $count || exit 1
    run_pair fold_send_release_each $count GLOO_AMD_FWD_RELEASE=each || exit 1
    run_pair unfused $count GLOO_AMD_FOLD_SEND=0 || exit 1
    run_pair copy_kernel256 $count GLOO_AMD_COPY=kernel GLOO_AMD_COPY_BLOCKS=256 || exit 1
  done
  tail -8 gpurun_out/latency_foldsend.jsonl
done
