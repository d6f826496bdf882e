#!/bin/bash
# tools/latency for 2 rank processes (HD fp32 sum), alternating labelled
# environment variants REPS times per count, so that variants are compared
# inside one session.  JSON lines into gpurun_out/latency_ab.jsonl.
#   tools/latency_ab.sh REPS "COUNT ..." LABEL[:VAR=VAL[,VAR=VAL...]] ...
# e.g. tools/latency_ab.sh 3 "256 262144" default each:GLOO_AMD_FWD_RELEASE=each
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run_pair() {  # label count env...
  local label=$1 count=$2; shift 2
  local d
  d=$(mktemp -d)
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 0 2 "file:$d" $count 600 >> gpurun_out/latency_ab.jsonl &
  local p0=$!
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 1 2 "file:$d" $count 600 > /dev/null &
  local p1=$!
  wait $p0 || return 1
  wait $p1 || return 1
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
