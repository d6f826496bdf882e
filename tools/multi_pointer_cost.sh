#!/bin/bash
# P processes of tools/multi_pointer_cost.py on GPU 0.  Usage:
#   tools/multi_pointer_cost.sh P N K ITERS
set -o pipefail
here=$(cd "$(dirname "$0")" && pwd)
d=$(mktemp -d)
P=$1; shift
pids=()
for ((r = 1; r < P; r++)); do
  timeout -k 10 ${BENCH_TIMEOUT:-200} python3 "$here/multi_pointer_cost.py" $r $P "$d" "$@" > /dev/null &
  pids+=($!)
done
timeout -k 10 ${BENCH_TIMEOUT:-200} python3 "$here/multi_pointer_cost.py" 0 $P "$d" "$@"
rc=$?
for p in "${pids[@]}"; do wait $p || rc=1; done
rm -rf "$d"
exit $rc
