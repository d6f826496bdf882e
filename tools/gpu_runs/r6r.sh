# GPUTEST_r05's case as a rate on round 5's own package (ff98d15, rebuilt unchanged)
set -o pipefail
mkdir -p gpurun_out/r6r
bash tools/gpu_session.sh \
 "400:r6r_r05:env GLOO_AMD_PKG_ROOT=$PWD/tools/ab/r05 python -u tools/bcube_threads_stress.py 200 > gpurun_out/r6r/r05_package.jsonl"
