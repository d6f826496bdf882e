#!/bin/bash
# HBM traffic per kernel of an HD allreduce (tools/latency, 2 rank
# processes): rank 0 under rocprofv3 --pmc, one counter per pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in separate passes), rank 1
# plain.  CSVs into gpurun_out/pmc_<LABEL>_<COUNTER>/.
#   tools/latency_pmc.sh LABEL COUNT
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
label=$1; count=$2
for counter in FETCH_SIZE WRITE_SIZE; do
  d=$(mktemp -d)
  timeout -s KILL 90 rocprofv3 --pmc $counter --output-format csv -d gpurun_out/pmc_${label}_${counter} -o p \
    -- ./tools/latency 0 2 "file:$d" $count 100 > /dev/null &
  p0=$!
  timeout -k 5 90 ./tools/latency 1 2 "file:$d" $count 100 > /dev/null &
  p1=$!
  wait $p0 || exit 1
  wait $p1 || exit 1
  rm -rf "$d"
done
