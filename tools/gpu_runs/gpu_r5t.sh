# round 5, GPU call t: 8-rank one-GPU rehearsal of the driver's N=8 bench on the VMM-only pool
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu --quick > gpurun_out/r5t_bench_n8_one_gpu_quick.json 2> gpurun_out/r5t_bench_n8_one_gpu_quick.err || { tail -30 gpurun_out/r5t_bench_n8_one_gpu_quick.err; exit 1; }
tail -c 300 gpurun_out/r5t_bench_n8_one_gpu_quick.json
mkdir -p gpurun_out/r5t_stress
timeout -k 10 150 python tools/stress.py 4 60 11 > gpurun_out/r5t_stress/p4_mesh.jsonl 2> gpurun_out/r5t_stress/p4_mesh.err || { tail -20 gpurun_out/r5t_stress/p4_mesh.err; exit 1; }
GLOO_AMD_MESH=0 timeout -k 10 120 python tools/stress.py 3 40 12 > gpurun_out/r5t_stress/p3_reference_route.jsonl 2> gpurun_out/r5t_stress/p3_reference_route.err || { tail -20 gpurun_out/r5t_stress/p3_reference_route.err; exit 1; }
tail -n 2 gpurun_out/r5t_stress/*.jsonl
