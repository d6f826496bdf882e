# round 5, GPU call ak: the interpreter's acquire scope after a wait (system vs agent), caller-stream latency
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/latency_ab.jsonl
LAT_ITERS=1000 timeout -k 10 300 bash tools/latency_ab.sh 3 "256 16384 262144 1048576" system agent:GLOO_AMD_INTERP_ACQUIRE=agent || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5ak_acquire_p2.jsonl
LAT_P=4 LAT_ITERS=1000 timeout -k 10 300 bash tools/latency_ab.sh 3 "256 262144" system agent:GLOO_AMD_INTERP_ACQUIRE=agent || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5ak_acquire_p4.jsonl
