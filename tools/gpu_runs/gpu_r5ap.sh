# round 5, GPU call ap: 2/4/8-rank one-GPU rehearsals of the bench on the final tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu > gpurun_out/r5ap_bench_n2.json 2> gpurun_out/r5ap_bench_n2.err || { tail -20 gpurun_out/r5ap_bench_n2.err; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 4 --steps 20 --warmup 5 --no-cpu --quick > gpurun_out/r5ap_bench_n4_quick.json 2> gpurun_out/r5ap_bench_n4_quick.err || { tail -20 gpurun_out/r5ap_bench_n4_quick.err; exit 1; }
timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu --quick > gpurun_out/r5ap_bench_n8_quick.json 2> gpurun_out/r5ap_bench_n8_quick.err || { tail -20 gpurun_out/r5ap_bench_n8_quick.err; exit 1; }
