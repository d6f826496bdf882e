#!/bin/bash
# Two processes of tools/transport_bench on GPU 0 (one JSON line per size on
# stdout).  Usage: tools/transport_bench.sh KIND [MIN_BYTES MAX_BYTES]
set -o pipefail
here=$(cd "$(dirname "$0")" && pwd)
d=$(mktemp -d)
timeout -k 10 ${BENCH_TIMEOUT:-240} "$here/transport_bench" 1 "$d" "$@" > /dev/null &
peer=$!
timeout -k 10 ${BENCH_TIMEOUT:-240} "$here/transport_bench" 0 "$d" "$@"
rc=$?
wait $peer
rc1=$?
rm -rf "$d"
[ $rc -eq 0 ] && [ $rc1 -eq 0 ]
