# one-pass multi-destination local broadcast
set -o pipefail
mkdir -p gpurun_out/r6g
bash tools/gpu_session.sh \
 "300:r6g_tests:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_collectives_gpu.py -k 'broadcast_one_pass or multi_pointer or threads_match_reference_golden or threads_repeated' tests/test_gloo_collectives.py tests/test_bridge.py" \
 "200:r6g_mp2:bash tools/multi_pointer_cost.sh 2 16777216 4 20 > gpurun_out/r6g/multi_pointer_p2.jsonl" \
 "200:r6g_mp4:bash tools/multi_pointer_cost.sh 4 4194304 4 20 > gpurun_out/r6g/multi_pointer_p4.jsonl"
