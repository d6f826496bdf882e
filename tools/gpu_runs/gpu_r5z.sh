# round 5, GPU call z: launch mode at mid sizes after the store changes: eager (default) vs graph replay
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/latency_ab.jsonl
LAT_ITERS=300 timeout -k 10 300 bash tools/latency_ab.sh 3 "1048576 4194304 16777216" default graph:GLOO_AMD_GRAPH=1 || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5z_mode_hd_p2.jsonl
LAT_P=4 LAT_ITERS=300 timeout -k 10 400 bash tools/latency_ab.sh 3 "1048576 4194304 16777216" default graph:GLOO_AMD_GRAPH=1 || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5z_mode_hd_p4.jsonl
