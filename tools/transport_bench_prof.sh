#!/bin/bash
# tools/transport_bench under rocprofv3 (rank 0 profiled, rank 1 plain): the
# kernels of the transport's device-to-device sends and their durations.
# Usage: tools/transport_bench_prof.sh OUTDIR KIND [MIN MAX]
set -o pipefail
here=$(cd "$(dirname "$0")" && pwd)
out=$1; shift
d=$(mktemp -d)
timeout -k 10 240 "$here/transport_bench" 1 "$d" "$@" > /dev/null &
peer=$!
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out" -o prof -- "$here/transport_bench" 0 "$d" "$@"
rc=$?
wait $peer
rc1=$?
rm -rf "$d"
[ $rc -eq 0 ] && [ $rc1 -eq 0 ]
