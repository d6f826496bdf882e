#!/bin/bash
# why the copy kernel loses to the blit as the copy-out of
# an HD call (a mesh result out of its inbox) while it wins in isolation.
# HD allreduce, 2 rank processes (tools/latency), COUNT fp32 per rank; the
# copy-out on the runtime's blit (default) and on the copy kernel
# (GLOO_AMD_COPY_OUT_BYTES=0, 256 workgroups); rank 0 under rocprofv3: one
# kernel-trace pass, then one pass per counter group (MI355X_MICROARCH.md:
# FETCH_SIZE and WRITE_SIZE in separate passes).  Then the same copy in
# isolation (tools/copy_engines.py, a fine-grained source as the inbox is).
# Output: gpurun_out/copyout_<engine>_<pass>/
#   tools/copy_out_pmc.sh COUNT
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
count=${1:-16777216}
root=$PWD
pair() {  # outdir env-assignments... -- profiler args...
  local out=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  local d
  d=$(mktemp -d)
  env "${envs[@]}" timeout -k 5 120 "$root/tools/latency" 1 2 "file:$d" $count 300 > /dev/null &
  local p1=$!
  (cd /tmp && env "${envs[@]}" timeout -s KILL 120 rocprofv3 "$@" -d "$root/gpurun_out/$out" -o p -- "$root/tools/latency" 0 2 "file:$d" $count 300 > "$root/gpurun_out/$out.json")
  local rc=$?
  wait $p1
  local rc1=$?
  rm -rf "$d"
  [ $rc -eq 0 ] && [ $rc1 -eq 0 ]
}
for engine in blit kernel; do
  if [ $engine = kernel ]; then E=(GLOO_AMD_COPY_OUT_BYTES=0 GLOO_AMD_COPY_OUT_BLOCKS=256); else E=(GLOO_AMD_NOP=1); fi
  pair copyout_${engine}_trace "${E[@]}" -- --kernel-trace --stats --output-format csv || exit 1
  pair copyout_${engine}_fetch "${E[@]}" -- --pmc FETCH_SIZE --output-format csv || exit 1
  pair copyout_${engine}_write "${E[@]}" -- --pmc WRITE_SIZE --output-format csv || exit 1
  pair copyout_${engine}_req "${E[@]}" -- --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_WRREQ_sum --output-format csv || exit 1
done
