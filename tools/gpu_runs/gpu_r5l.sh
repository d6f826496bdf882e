# round 5, GPU call l: new golden-coverage GPU cases, smoke, bench N=1 (+ rocprof), copy-out PMC
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 300 python -u -m pytest tests/test_newstyle_gpu.py tests/test_reduce_gpu.py -k "P12 or defect" -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5l_pytest_new.log 2>&1 || { tail -30 gpurun_out/r5l_pytest_new.log; exit 1; }
tail -2 gpurun_out/r5l_pytest_new.log
step smoke
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5l_smoke.log 2>&1 || { tail -30 gpurun_out/r5l_smoke.log; exit 1; }
tail -1 gpurun_out/r5l_smoke.log
step bench
timeout -k 10 600 python -u bench.py > gpurun_out/r5l_bench_n1.json 2> gpurun_out/r5l_bench_n1.err || { tail -30 gpurun_out/r5l_bench_n1.err; exit 1; }
cut -c1-400 gpurun_out/r5l_bench_n1.json | tail -1
step rocprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5l_prof -o p -- python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r5l_bench_k20_rocprof.json 2> gpurun_out/r5l_bench_k20_rocprof.err || { tail -30 gpurun_out/r5l_bench_k20_rocprof.err; exit 1; }
step copyout
timeout -k 10 500 bash tools/copy_out_pmc.sh 16777216 > gpurun_out/r5l_copyout.log 2>&1 || { tail -30 gpurun_out/r5l_copyout.log; exit 1; }
step done
