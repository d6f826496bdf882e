# round 5, GPU call p: store flavours of a collective's local results (copy-out default now plain kernel; fold dst)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/latency_ab.jsonl
OLD="GLOO_AMD_COPY_OUT_BYTES=18446744073709551615"
LAT_ITERS=300 timeout -k 10 300 bash tools/latency_ab.sh 3 "4194304 16777216" old:$OLD new foldplain:GLOO_AMD_FOLD_STORE=plain || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5p_store_hd_p2.jsonl
LAT_P=4 LAT_ITERS=300 timeout -k 10 400 bash tools/latency_ab.sh 3 "4194304 16777216 67108864" old:$OLD new foldplain:GLOO_AMD_FOLD_STORE=plain || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5p_store_hd_p4.jsonl
LATENCY_ALGO=ring_chunked LAT_P=4 LAT_ITERS=200 timeout -k 10 400 bash tools/latency_ab.sh 3 "4194304 16777216 67108864" old:$OLD new foldplain:GLOO_AMD_FOLD_STORE=plain || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5p_store_ring_p4.jsonl
