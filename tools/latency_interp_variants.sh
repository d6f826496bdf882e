#!/bin/bash
# tools/latency (2 rank processes, HD fp32) at 4 and 16 MiB per rank: graph
# replay against the sliced interpreter, for each interpreter build of
# tools/build_interp_variants.sh and several slice geometries.  JSON lines
# into gpurun_out/latency_iv.jsonl.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run_pair() {  # label count env...
  local label=$1 count=$2; shift 2
  local d
  d=$(mktemp -d)
  env "$@" LATENCY_LABEL=$label timeout -k 5 60 ./tools/latency 0 2 "file:$d" $count 300 >> gpurun_out/latency_iv.jsonl &
  local p0=$!
  env "$@" LATENCY_LABEL=$label timeout -k 5 60 ./tools/latency 1 2 "file:$d" $count 300 > /dev/null &
  local p1=$!
  wait $p0 || return 1
  wait $p1 || return 1
  rm -rf "$d"
}
for count in 1048576 4194304; do
  run_pair graph $count GLOO_AMD_GRAPH=1 GLOO_AMD_INTERP=0 || exit 1
  for v in default $(ls tools/interp_variants); do
    lp=""; [ $v != default ] && lp="LD_LIBRARY_PATH=$PWD/tools/interp_variants/$v"
    for geo in 64:32768 32:65536 128:32768 64:65536 128:65536 256:32768 256:65536; do
      ms=${geo%%:*}; sb=${geo##*:}
      run_pair "$v/${ms}x$((sb/1024))k" $count $lp GLOO_AMD_INTERP_MAX_SLICES=$ms GLOO_AMD_INTERP_SLICE_BYTES=$sb || exit 1
    done
    echo "$count $v done"
  done
done
