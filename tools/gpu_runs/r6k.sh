# the stale-line mechanism on one buffer
set -o pipefail
mkdir -p gpurun_out/r6k
bash tools/gpu_session.sh \
 "120:r6k_stale4k:./tools/stale_line_probe 3000 4096 > gpurun_out/r6k/stale_line_4k.jsonl" \
 "120:r6k_stale64k:./tools/stale_line_probe 2000 65536 > gpurun_out/r6k/stale_line_64k.jsonl"
