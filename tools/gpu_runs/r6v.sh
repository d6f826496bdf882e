# host staging pipelined again in >= 16 MiB pieces: parity and rates
set -o pipefail
mkdir -p gpurun_out/r6v
bash tools/gpu_session.sh \
 "300:r6v_staged:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_staged_gpu.py" \
 "300:r6v_bench:python -u bench.py --steps 200 --no-cpu > gpurun_out/r6v/bench_n1_host_staged.json"
