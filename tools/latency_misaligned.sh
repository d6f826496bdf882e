#!/bin/bash
# Interpreter messages at misaligned offsets (VERDICT r1 #5b): HD allreduce
# with 2 rank processes on one GPU, element counts whose halves start on a
# 16-byte boundary (262144, 16384) against counts whose halves do not
# (262147, 16387: every peer piece and fold operand 4 bytes off).  Since
# round 2 the interpreter moves misaligned operands in 16-byte packets
# (buffer soffset), so the two should cost the same.  JSON lines into
# gpurun_out/latency_misaligned.jsonl.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/latency_misaligned.jsonl
run_pair() {  # label count env...
  local label=$1 count=$2; shift 2
  local d
  d=$(mktemp -d)
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 0 2 "file:$d" $count 2000 >> $out &
  local p0=$!
  env "$@" LATENCY_LABEL=$label timeout -k 5 120 ./tools/latency 1 2 "file:$d" $count 2000 >> $out &
  local p1=$!
  wait $p0 || return 1
  wait $p1 || return 1
  rm -rf "$d"
}
for rep in 1 2; do
  for count in 16384 16387 262144 262147; do
    run_pair "rep$rep" $count || exit 1
  done
done
cat $out
