# round 5, GPU call at: the sliced interpreter at mid sizes with more slices (caller-stream latency)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/latency_ab.jsonl
LAT_ITERS=300 timeout -k 10 300 bash tools/latency_ab.sh 3 "1048576 4194304" default s64:GLOO_AMD_INTERP_MAX_SLICES=64 s128:GLOO_AMD_INTERP_MAX_SLICES=128 s128w:GLOO_AMD_INTERP_MAX_SLICES=128,GLOO_AMD_INTERP_SLICE_MAX_BYTES=131072 || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5at_slices_p2.jsonl
LAT_P=4 LAT_ITERS=300 timeout -k 10 300 bash tools/latency_ab.sh 3 "1048576 4194304" default s64:GLOO_AMD_INTERP_MAX_SLICES=64 s128:GLOO_AMD_INTERP_MAX_SLICES=128 || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5at_slices_p4.jsonl
