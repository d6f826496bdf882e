# the whole GPU suite on the round-6 tree after the transport, pool and broadcast changes; smoke; default bench
set -o pipefail
mkdir -p gpurun_out/r6o
bash tools/gpu_session.sh \
 "900:r6o_pytest_gpu_all:python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests" \
 "200:r6o_smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")'" \
 "300:r6o_bench:python -u bench.py > gpurun_out/r6o/bench_n1.json"
