# AllreduceBcube / CudaAllreduceBcube on the GPU: golden thread and process cases, the Gloo bridge program
set -o pipefail
mkdir -p gpurun_out/r6y
bash tools/gpu_session.sh \
 "600:r6y_bcube:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bcube_gpu.py" \
 "600:r6y_bridge:python -u -m pytest -x -v --timeout 560 --timeout-method thread tests/test_bridge.py -m gpu"
