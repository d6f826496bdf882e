# round 5, GPU call af: the GPU suite and a 2-rank bench rehearsal with the interpreter's done flag
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider --durations=25 > gpurun_out/r5af_pytest_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r5af_pytest_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu > gpurun_out/r5af_bench_n2_one_gpu.json 2> gpurun_out/r5af_bench_n2_one_gpu.err || { tail -20 gpurun_out/r5af_bench_n2_one_gpu.err; exit 1; }
