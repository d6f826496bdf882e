#!/bin/bash
# Run tools/pingpong for every (flag placement, kernel shape) pair with two
# rank processes; one JSON line per rank and pair into gpurun_out/pingpong.jsonl.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for place in host device; do
  for shape in split fused; do
    d=$(mktemp -d)
    timeout -k 5 60 ./tools/pingpong 0 "file:$d" $place $shape 2000 5 >> gpurun_out/pingpong.jsonl &
    p0=$!
    timeout -k 5 60 ./tools/pingpong 1 "file:$d" $place $shape 2000 5 >> gpurun_out/pingpong.jsonl &
    p1=$!
    wait $p0; wait $p1
    rm -rf "$d"
  done
done
cat gpurun_out/pingpong.jsonl
