# mixed-collective stress with AllreduceBcube in the mix: 4 and 8 ranks on the default routes, 4 ranks on the
# reference routes (every result checked exactly; one JSON line per rank)
set -o pipefail
mkdir -p gpurun_out/r6ac
bash tools/gpu_session.sh \
 "200:r6ac_p4:python -u tools/stress.py 4 60 21 > gpurun_out/r6ac/stress_p4.jsonl" \
 "240:r6ac_p8:python -u tools/stress.py 8 60 22 > gpurun_out/r6ac/stress_p8.jsonl" \
 "200:r6ac_p4_ref:GLOO_AMD_MESH=0 python -u tools/stress.py 4 45 23 > gpurun_out/r6ac/stress_p4_mesh0.jsonl"
