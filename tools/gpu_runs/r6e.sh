# dma-buf ranges instead of hipIpc in the transport
set -o pipefail
mkdir -p gpurun_out/r6e
bash tools/gpu_session.sh \
 "90:r6e_probe_big:./tools/dmabuf_probe 2684354560 > gpurun_out/r6e/dmabuf_probe_2p5gib.jsonl" \
 "400:r6e_transport:python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_transport_gpu.py tests/test_gloo_transport.py tests/test_ipc_pool_gpu.py" \
 "300:r6e_tbench:bash tools/transport_bench.sh device > gpurun_out/r6e/tbench_device.jsonl"
