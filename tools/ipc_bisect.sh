#!/bin/bash
# DIAGNOSIS ONLY: tools/ipc_bisect.py over a matrix of first-executor settings.
set -o pipefail
export GLOO_AMD_RING_MESH=0 GLOO_AMD_IPC_POOL=${POOL:-0}
out=${OUT:-gpurun_out/ipc_bisect.jsonl}
: > "$out"
while read -r first runs prof; do
  [ -z "$first" ] && continue
  echo "case first=$first runs=$runs profile=$prof"
  timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) tools/ipc_bisect.py --first "$first" --runs "$runs" --profile "$prof" \
    2>>"${out%.jsonl}.err" | grep '^{' | tee -a "$out" | cut -c1-200 || exit 1
done <<CASES
${CASES:-COPY=memcpy 3 0
COPY=memcpy,GRAPH=0 3 0
COPY=memcpy 1 0
COPY=kernel 3 0
COPY=memcpy 3 1
COPY=memcpy 3 2}
CASES
