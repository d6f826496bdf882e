# final tree (host staging pipelined in >= 16 MiB pieces): staged parity, the whole GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out/r6w
bash tools/gpu_session.sh \
 "300:r6w_staged:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_staged_gpu.py" \
 "900:r6w_pytest_gpu_all:python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests" \
 "200:r6w_smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")'" \
 "300:r6w_bench:python -u bench.py > gpurun_out/r6w/bench_n1.json"
