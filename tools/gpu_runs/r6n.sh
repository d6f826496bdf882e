# does a stream / event synchronise wait for a slow host function?
set -o pipefail
mkdir -p gpurun_out/r6n
bash tools/gpu_session.sh \
 "120:r6n_hostfn:./tools/hostfn_order_probe 100 2 50 > gpurun_out/r6n/hostfn_order.jsonl"
