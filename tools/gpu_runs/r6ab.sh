# AllreduceBcube with its derived mesh plan as the default for 2 <= P <= 8 (reference route as the fallback and
# under GLOO_AMD_MESH=0): bcube goldens, custom-op cases, the stress runs, the Gloo bridge program
set -o pipefail
mkdir -p gpurun_out/r6ab
bash tools/gpu_session.sh \
 "600:r6ab_bcube:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bcube_gpu.py tests/test_custom_op_gpu.py" \
 "600:r6ab_stress:python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_collectives_gpu.py -k stress" \
 "600:r6ab_bridge:python -u -m pytest -x -v --timeout 560 --timeout-method thread tests/test_bridge.py -m gpu"
