# round 5, GPU call o: copy-out on the copy kernel with plain stores, sizes and rank counts
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/latency_ab.jsonl
K="GLOO_AMD_COPY_OUT_BYTES=0,GLOO_AMD_PLAIN_COPY_STORE=plain"
LAT_ITERS=300 timeout -k 10 300 bash tools/latency_ab.sh 3 "262144 1048576 67108864" blit kplain:$K || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5o_copyout_plain_p2.jsonl
LAT_P=4 LAT_ITERS=300 timeout -k 10 400 bash tools/latency_ab.sh 3 "1048576 4194304 16777216 67108864" blit kplain:$K || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5o_copyout_plain_p4.jsonl
