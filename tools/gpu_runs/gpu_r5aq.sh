# round 5, GPU call aq: the P = 8 process batches with 4 (default) and 1 hardware queue per process
set -o pipefail
mkdir -p gpurun_out
for q in 4 1 4 1; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u -m pytest tests/test_collectives_gpu.py -k "P8 and (graph_replay or sliced or host_workspace or fold_send)" -m gpu -q --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/r5aq_q${q}.log 2>&1 || { tail -20 gpurun_out/r5aq_q${q}.log; exit 1; }
  echo "queues=$q $(tail -1 gpurun_out/r5aq_q${q}.log)"
done
