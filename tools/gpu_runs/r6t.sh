# N = 2 and N = 4 bench rehearsals (ranks share the one GPU) on the final tree
set -o pipefail
mkdir -p gpurun_out/r6t
bash tools/gpu_session.sh \
 "600:r6t_bench2:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r6t/bench_n2_one_gpu.json" \
 "700:r6t_bench4:python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 20 --warmup 5 > gpurun_out/r6t/bench_n4_one_gpu.json"
