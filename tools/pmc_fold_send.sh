#!/bin/bash
# Attribute fold_send_kernel's HBM reads: HD fp32 allreduce,
# 2 rank processes on one GPU (tools/latency), rank 0 under rocprofv3 --pmc,
# one counter set per pass (MI355X_MICROARCH.md: TCC holds 4 counters;
# FETCH_SIZE alone uses 3), per variant:
#   fused     the default (fold + forward in one launch)
#   unfused   GLOO_AMD_FOLD_SEND=0 (a pure fold, then the copy kernel)
#   coarse    GLOO_AMD_ARENA=coarse (inboxes in coarse-grained HBM)
# CSVs into gpurun_out/pmcfs_<variant>_<set>/; summarise with
# tools/pmc_fold_send.py.   tools/pmc_fold_send.sh COUNT [ITERS]
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
count=$1; iters=${2:-100}
sets=("FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum"
      "TCC_EA0_RD_UNCACHED_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum")
names=(fetch write rdreq uncached)
for variant in fused unfused coarse; do
  case $variant in
    fused) envs=();;
    unfused) envs=(GLOO_AMD_FOLD_SEND=0);;
    coarse) envs=(GLOO_AMD_ARENA=coarse);;
  esac
  for k in "${!sets[@]}"; do
    d=$(mktemp -d)
    env "${envs[@]}" timeout -s KILL 90 rocprofv3 --pmc ${sets[$k]} --output-format csv \
      -d gpurun_out/pmcfs_${variant}_${names[$k]} -o p -- ./tools/latency 0 2 "file:$d" $count $iters > /dev/null &
    p0=$!
    env "${envs[@]}" timeout -k 5 90 ./tools/latency 1 2 "file:$d" $count $iters > /dev/null &
    p1=$!
    wait $p0 || exit 1
    wait $p1 || exit 1
    rm -rf "$d"
  done
done
python3 tools/pmc_fold_send.py gpurun_out $count | tee gpurun_out/pmc_fold_send_summary.json
