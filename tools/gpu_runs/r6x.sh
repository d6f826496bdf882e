# host-staged choices interleaved (7 rounds); final-tree rocprof of the bench's config-2 sections and PMC traffic
set -o pipefail
mkdir -p gpurun_out/r6x
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_session.sh \
 "300:r6x_staged_sweep:python -u tools/host_staged_sweep.py --rounds 7 > gpurun_out/r6x/host_staged_sweep.jsonl" \
 "400:r6x_prof:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6x/prof -o r6x -- python3 bench.py --no-cpu --no-host-staged > gpurun_out/r6x/bench_n1_under_rocprof.json" \
 "120:r6x_fetch:timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r6x/pmc_fetch -o f -- python3 bench.py --steps 25 --warmup 0 --no-cpu --no-host-staged" \
 "120:r6x_write:timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r6x/pmc_write -o w -- python3 bench.py --steps 25 --warmup 0 --no-cpu --no-host-staged" \
 "200:r6x_bench_k20:for i in 1 2 3; do python -u bench.py --steps 20 --warmup 5 --no-cpu --no-host-staged; done > gpurun_out/r6x/bench_k20_x3.jsonl"
