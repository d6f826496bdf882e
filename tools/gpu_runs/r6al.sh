# the driver's bench command on a fresh box, final tree (twice, the second without the CPU legs)
set -o pipefail
mkdir -p gpurun_out/r6al
bash tools/gpu_session.sh \
 "300:r6al_bench:python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6al/bench_n1.json" \
 "200:r6al_bench2:python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-host-staged > gpurun_out/r6al/bench_n1_again.json"
