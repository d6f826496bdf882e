# round 5, GPU call n: copy-out engine and store flavour A/B interleaved
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/latency_ab.jsonl
K="GLOO_AMD_COPY_OUT_BYTES=0,GLOO_AMD_COPY_OUT_BLOCKS=256"
timeout -k 10 500 bash tools/latency_ab.sh 4 "16777216 4194304" blit knt:$K kwt:$K,GLOO_AMD_PLAIN_COPY_STORE=wt kplain:$K,GLOO_AMD_PLAIN_COPY_STORE=plain || exit 1
mv gpurun_out/latency_ab.jsonl gpurun_out/r5n_copyout_store_ab_p2.jsonl
