# the whole GPU suite after the stress-line fix; smoke; default bench
set -o pipefail
mkdir -p gpurun_out/r6p
bash tools/gpu_session.sh \
 "900:r6p_pytest_gpu_all:python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests" \
 "200:r6p_smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")'" \
 "300:r6p_bench:python -u bench.py > gpurun_out/r6p/bench_n1.json"
