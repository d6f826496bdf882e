# round 5, GPU call y: PMC traffic of the headline kernel on the round-5 build (separate FETCH / WRITE passes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r5y_fetch -o p -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-host-staged > gpurun_out/r5y_fetch.json 2> gpurun_out/r5y_fetch.err || { tail -20 gpurun_out/r5y_fetch.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r5y_write -o p -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-host-staged > gpurun_out/r5y_write.json 2> gpurun_out/r5y_write.err || { tail -20 gpurun_out/r5y_write.err; exit 1; }
ls gpurun_out/r5y_fetch gpurun_out/r5y_write
