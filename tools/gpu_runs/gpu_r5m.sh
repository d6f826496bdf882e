# round 5, GPU call m: copy-out engine A/B interleaved inside one session
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/latency_ab.jsonl
timeout -k 10 400 bash tools/latency_ab.sh 4 "4194304 16777216" blit kernel256:GLOO_AMD_COPY_OUT_BYTES=0,GLOO_AMD_COPY_OUT_BLOCKS=256 kernel1024:GLOO_AMD_COPY_OUT_BYTES=0,GLOO_AMD_COPY_OUT_BLOCKS=1024 || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5m_copyout_ab_p2.jsonl
LAT_P=4 timeout -k 10 400 bash tools/latency_ab.sh 3 "16777216" blit kernel256:GLOO_AMD_COPY_OUT_BYTES=0,GLOO_AMD_COPY_OUT_BLOCKS=256 || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5m_copyout_ab_p4.jsonl
