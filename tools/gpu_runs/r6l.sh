# does a stream host function wait for the kernels before it?
set -o pipefail
mkdir -p gpurun_out/r6l
bash tools/gpu_session.sh \
 "120:r6l_hostfn:./tools/hostfn_order_probe 300 2 10 50 200 > gpurun_out/r6l/hostfn_order.jsonl"
