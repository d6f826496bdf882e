#!/bin/bash
# tools/latency for LAT_P (default 2) rank processes (HD fp32 sum), alternating labelled
# environment variants REPS times per count, so that variants are compared
# inside one session.  JSON lines into gpurun_out/latency_ab.jsonl.
#   tools/latency_ab.sh REPS "COUNT ..." LABEL[:VAR=VAL[,VAR=VAL...]] ...
# e.g. tools/latency_ab.sh 3 "256 262144" default each:GLOO_AMD_FWD_RELEASE=each
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
P=${LAT_P:-2}          # rank processes (all on this GPU)
ITERS=${LAT_ITERS:-600}
run_pair() {  # label count env...
  local label=$1 count=$2; shift 2
  local d pids=() r
  d=$(mktemp -d)
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 0 $P "file:$d" $count $ITERS >> gpurun_out/latency_ab.jsonl &
  pids+=($!)
  for r in $(seq 1 $((P - 1))); do
    env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency $r $P "file:$d" $count $ITERS > /dev/null &
    pids+=($!)
  done
  for r in "${pids[@]}"; do wait $r || return 1; done
  rm -rf "$d"
}
reps=$1; counts=$2; shift 2
for count in $counts; do
  for rep in $(seq "$reps"); do
    for spec in "$@"; do
      label=${spec%%:*}
      envs=()
      if [ "$spec" != "$label" ]; then IFS=',' read -ra envs <<< "${spec#*:}"; fi
      run_pair "$label" "$count" "${envs[@]}" || exit 1
    done
  done
done
wc -l gpurun_out/latency_ab.jsonl
