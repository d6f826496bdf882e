# the whole GPU suite with AllreduceBcube (48 cases), the 4-rank stress run and the bcube custom-op cases; smoke; default bench
set -o pipefail
mkdir -p gpurun_out/r6z
bash tools/gpu_session.sh \
 "900:r6z_pytest_gpu_all:python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests" \
 "200:r6z_smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")'" \
 "300:r6z_bench:python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6z/bench_n1.json"
