# round 5, GPU call u: store flavour of the reference routes' REDUCE steps (GLOO_AMD_MESH=0)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/latency_ab.jsonl
LAT_ITERS=300 timeout -k 10 300 bash tools/latency_ab.sh 3 "1048576 4194304 16777216" nt:GLOO_AMD_MESH=0 plain:GLOO_AMD_MESH=0,GLOO_AMD_REDUCE_STORE=plain || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5u_reduce_store_hd_p2.jsonl
LAT_P=4 LAT_ITERS=300 timeout -k 10 400 bash tools/latency_ab.sh 3 "4194304 16777216 67108864" nt:GLOO_AMD_MESH=0 plain:GLOO_AMD_MESH=0,GLOO_AMD_REDUCE_STORE=plain || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5u_reduce_store_hd_p4.jsonl
LATENCY_ALGO=ring_chunked LAT_P=4 LAT_ITERS=200 timeout -k 10 400 bash tools/latency_ab.sh 3 "4194304 16777216 67108864" nt:GLOO_AMD_RING_MESH=0 plain:GLOO_AMD_RING_MESH=0,GLOO_AMD_REDUCE_STORE=plain || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5u_reduce_store_ring_p4.jsonl
