#!/bin/bash
# Kernel trace of one small-allreduce latency run (tools/latency, 2 rank
# processes, 1 KiB HD, default launch mode = the one-launch interpreter):
# rank 0 under rocprofv3 --kernel-trace --stats, rank 1 plain.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
d=$(mktemp -d)
count=${1:-256}
export TMPDIR=/tmp
timeout -k 5 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_latency -o lat \
  -- ./tools/latency 0 2 "file:$d" $count 1000 > gpurun_out/latency_prof_rank0.json &
p0=$!
timeout -k 5 120 ./tools/latency 1 2 "file:$d" $count 1000 > gpurun_out/latency_prof_rank1.json &
p1=$!
wait $p0 || exit 1
wait $p1 || exit 1
rm -rf "$d"
find gpurun_out/prof_latency -name "*kernel_stats.csv" -exec cat {} \;
