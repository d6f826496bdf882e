# A/B: plain against nt stores in the executor's multi-source folds (LOCAL_REDUCE, FOLD)
set -o pipefail
mkdir -p gpurun_out/r6i
NT="GLOO_AMD_LIB=$GRAFT_REPO_ROOT/tools/ab/libgloo_amd_ntfold.so"
bash tools/gpu_session.sh \
 "150:r6i_p2a:bash tools/multi_pointer_cost.sh 2 16777216 4 30 >> gpurun_out/r6i/plain_p2.jsonl" \
 "150:r6i_p2b:env $NT bash tools/multi_pointer_cost.sh 2 16777216 4 30 >> gpurun_out/r6i/nt_p2.jsonl" \
 "150:r6i_p4a:bash tools/multi_pointer_cost.sh 4 4194304 4 30 >> gpurun_out/r6i/plain_p4.jsonl" \
 "150:r6i_p4b:env $NT bash tools/multi_pointer_cost.sh 4 4194304 4 30 >> gpurun_out/r6i/nt_p4.jsonl" \
 "150:r6i_p2c:bash tools/multi_pointer_cost.sh 2 16777216 4 30 >> gpurun_out/r6i/plain_p2.jsonl" \
 "150:r6i_p2d:env $NT bash tools/multi_pointer_cost.sh 2 16777216 4 30 >> gpurun_out/r6i/nt_p2.jsonl" \
 "150:r6i_p4c:bash tools/multi_pointer_cost.sh 4 4194304 4 30 >> gpurun_out/r6i/plain_p4.jsonl" \
 "150:r6i_p4d:env $NT bash tools/multi_pointer_cost.sh 4 4194304 4 30 >> gpurun_out/r6i/nt_p4.jsonl" \
 "300:r6i_tests:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_reduce_gpu.py tests/test_collectives_gpu.py -k 'multi or golden or fold or graph or interp'"
