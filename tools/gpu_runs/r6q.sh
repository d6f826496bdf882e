# GPUTEST_r05's case as an A/B rate: coarse-grained inbox (round-5 rule) against the product
set -o pipefail
mkdir -p gpurun_out/r6q
bash tools/gpu_session.sh \
 "300:r6q_coarse:env GLOO_AMD_LIB=$PWD/tools/ab/libgloo_amd_coarse_inbox.so python -u tools/bcube_threads_stress.py 150 > gpurun_out/r6q/coarse.jsonl" \
 "300:r6q_fine:python -u tools/bcube_threads_stress.py 150 > gpurun_out/r6q/fine.jsonl"
