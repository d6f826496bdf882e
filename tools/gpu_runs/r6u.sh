# bench relaunch tests after the stdout change
set -o pipefail
mkdir -p gpurun_out/r6u
bash tools/gpu_session.sh \
 "500:r6u_benchtests:python -u -m pytest -x -v --timeout 420 --timeout-method thread tests/test_bench_gpu.py" \
 "400:r6u_bench2:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r6u/bench_n2_one_gpu.json"
