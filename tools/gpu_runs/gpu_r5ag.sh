# round 5, GPU call ah: the done signal behind eager / replayed own-stream runs
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/latency_ab.jsonl
LAT_ITERS=300 timeout -k 10 300 bash tools/latency_ab.sh 3 "256 262144 4194304 16777216" spin:LATENCY_OWN_STREAM=1 sync:LATENCY_OWN_STREAM=1,GLOO_AMD_DONE_SPIN=0 ref_spin:LATENCY_OWN_STREAM=1,GLOO_AMD_MESH=0 ref_sync:LATENCY_OWN_STREAM=1,GLOO_AMD_MESH=0,GLOO_AMD_DONE_SPIN=0 || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5ah_done_spin_eager_p2.jsonl
LAT_P=4 LAT_ITERS=200 timeout -k 10 300 bash tools/latency_ab.sh 3 "4194304 16777216" spin:LATENCY_OWN_STREAM=1 sync:LATENCY_OWN_STREAM=1,GLOO_AMD_DONE_SPIN=0 || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5ah_done_spin_eager_p4.jsonl
