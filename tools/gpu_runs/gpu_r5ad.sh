# round 5, GPU call ad: the interpreter's done flag (own-stream runs spin on it) against synchronising the stream
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/latency_ab.jsonl
LAT_ITERS=1000 timeout -k 10 300 bash tools/latency_ab.sh 3 "256 16384 262144 1048576" spin:LATENCY_OWN_STREAM=1 sync:LATENCY_OWN_STREAM=1,GLOO_AMD_DONE_SPIN=0 caller || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5ad_done_spin_p2.jsonl
LAT_P=4 LAT_ITERS=1000 timeout -k 10 300 bash tools/latency_ab.sh 3 "256 262144" spin:LATENCY_OWN_STREAM=1 sync:LATENCY_OWN_STREAM=1,GLOO_AMD_DONE_SPIN=0 || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5ad_done_spin_p4.jsonl
