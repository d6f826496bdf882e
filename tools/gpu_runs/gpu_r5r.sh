# round 5, GPU call r: one-GPU rehearsals of the multi-rank bench (N=2 full collective section, N=4 quick)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu > gpurun_out/r5r_bench_n2_one_gpu.json 2> gpurun_out/r5r_bench_n2_one_gpu.err || { tail -20 gpurun_out/r5r_bench_n2_one_gpu.err; exit 1; }
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 20 --warmup 5 --no-cpu --quick > gpurun_out/r5r_bench_n4_one_gpu_quick.json 2> gpurun_out/r5r_bench_n4_one_gpu_quick.err || { tail -20 gpurun_out/r5r_bench_n4_one_gpu_quick.err; exit 1; }
