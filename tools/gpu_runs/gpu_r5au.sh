# round 5, GPU call au: the GPU suite, smoke and the default N=1 bench on the tree of the round's end
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider --durations=25 > gpurun_out/r5au_pytest_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5au_pytest_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5au_smoke.log 2>&1 || { tail -20 gpurun_out/r5au_smoke.log; exit 1; }
tail -1 gpurun_out/r5au_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r5au_bench_n1.json 2> gpurun_out/r5au_bench_n1.err || { tail -20 gpurun_out/r5au_bench_n1.err; exit 1; }
cut -c1-300 gpurun_out/r5au_bench_n1.json | tail -1
