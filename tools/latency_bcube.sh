#!/bin/bash
# tools/latency with P rank processes on the box's GPU(s): AllreduceBcube (base 2, base 4 at P = 4, and on the
# reference route) against halving-doubling, 1 KiB .. 16 MiB per rank.  JSON lines (one per rank) into
# gpurun_out/latency_bcube.jsonl; LATENCY_LABEL names the variant.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/latency_bcube.jsonl
run_ranks() {  # P label count env...
  local P=$1 label=$2 count=$3; shift 3
  local d pids=()
  d=$(mktemp -d)
  for ((r = 0; r < P; r++)); do
    env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency $r $P "file:$d" $count 1000 >> $out &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait $p || return 1; done
  rm -rf "$d"
}
for P in 2 4; do
  for count in 256 16384 262144 1048576 4194304; do
    run_ranks $P hd $count LATENCY_ALGO=halving_doubling || exit 1
    run_ranks $P bcube_b2 $count LATENCY_ALGO=bcube LATENCY_BASE=2 || exit 1
    run_ranks $P bcube_b2_reference_route $count LATENCY_ALGO=bcube LATENCY_BASE=2 GLOO_AMD_MESH=0 || exit 1
    if [ $P -eq 4 ]; then run_ranks $P bcube_b4 $count LATENCY_ALGO=bcube LATENCY_BASE=4 || exit 1; fi
  done
done
