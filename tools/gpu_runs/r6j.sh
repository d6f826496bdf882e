# the big-arena variants (gpu_extended) on the best-fit pool; the new transport realloc case
set -o pipefail
bash tools/gpu_session.sh \
 "200:r6j_transport:python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_transport_gpu.py -k 'realloc or resend or 2p5gib'" \
 "600:r6j_extended:env GLOO_AMD_GPU_EXTENDED=1 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu_extended tests"
