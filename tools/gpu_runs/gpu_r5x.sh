# round 5, GPU call x: the headline bench under rocprofv3 with only the config-2 kernel sections (the
# kernel-stats average is then the timed kernel's), 1000 steps like the default run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5x_prof -o p -- python3 bench.py --steps 1000 --warmup 50 --no-cpu --no-host-staged > gpurun_out/r5x_bench_k1000_rocprof.json 2> gpurun_out/r5x_bench_k1000_rocprof.err || { tail -20 gpurun_out/r5x_bench_k1000_rocprof.err; exit 1; }
tail -c 400 gpurun_out/r5x_bench_k1000_rocprof.json
