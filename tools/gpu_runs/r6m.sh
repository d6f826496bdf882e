# the thread route ordering around a busy stream
set -o pipefail
mkdir -p gpurun_out/r6m
bash tools/gpu_session.sh \
 "120:r6m_busy256:./tools/stale_busy_probe 3000 256 > gpurun_out/r6m/stale_busy_256.jsonl" \
 "120:r6m_busy64k:./tools/stale_busy_probe 1000 65536 > gpurun_out/r6m/stale_busy_64k.jsonl"
