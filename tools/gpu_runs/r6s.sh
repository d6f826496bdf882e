# final-tree profiles: the bench's config-2 sections under rocprofv3 --kernel-trace --stats, and the kernel's
# HBM traffic from FETCH_SIZE / WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md HBM section)
set -o pipefail
mkdir -p gpurun_out/r6s
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_session.sh \
 "400:r6s_prof:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6s/prof -o r6s -- python3 bench.py --no-cpu --no-host-staged > gpurun_out/r6s/bench_n1_under_rocprof.json" \
 "120:r6s_fetch:timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r6s/pmc_fetch -o f -- python3 bench.py --steps 25 --warmup 0 --no-cpu --no-host-staged" \
 "120:r6s_write:timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r6s/pmc_write -o w -- python3 bench.py --steps 25 --warmup 0 --no-cpu --no-host-staged"
