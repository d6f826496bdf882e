# the N > 1 bench path on the final tree (torchrun, every rank on the one GPU; K = 20): N = 2 and N = 4
set -o pipefail
mkdir -p gpurun_out/r6ah
bash tools/gpu_session.sh \
 "500:r6ah_n2:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r6ah/bench_n2_one_gpu.json" \
 "700:r6ah_n4:python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 4 --steps 20 --warmup 5 > gpurun_out/r6ah/bench_n4_one_gpu.json"
