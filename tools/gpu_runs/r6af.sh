# final tree (product kernel loads stream by stream): the whole GPU suite, smoke, driver-shaped benches,
# the bench's config-2 sections under rocprofv3 --kernel-trace --stats, PMC traffic in separate passes
set -o pipefail
mkdir -p gpurun_out/r6af
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_session.sh \
 "200:r6af_ab:python -u tools/tune/hbm_ceiling.py --lib libceiling_pre.so --steps 500 --reps 10 --only product_reduce_inplace > gpurun_out/r6af/load_order_ab_64mib.jsonl" \
 "900:r6af_pytest_gpu_all:python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests" \
 "200:r6af_smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")'" \
 "300:r6af_bench:python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6af/bench_n1.json" \
 "200:r6af_bench_k20:for i in 1 2 3 4 5; do python -u bench.py --steps 20 --warmup 5 --no-cpu --no-host-staged; done > gpurun_out/r6af/bench_k20_x5.jsonl" \
 "400:r6af_prof:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6af/prof -o r6af -- python3 bench.py --no-cpu --no-host-staged > gpurun_out/r6af/bench_n1_under_rocprof.json" \
 "120:r6af_fetch:timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r6af/pmc_fetch -o f -- python3 bench.py --steps 25 --warmup 0 --no-cpu --no-host-staged" \
 "120:r6af_write:timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r6af/pmc_write -o w -- python3 bench.py --steps 25 --warmup 0 --no-cpu --no-host-staged"
