# round 5, GPU call as: collectives tests + a 2-rank rehearsal with the adaptive completion spin
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_collectives_gpu.py tests/test_newstyle_gpu.py tests/test_gloo_collectives.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5as_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5as_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu > gpurun_out/r5as_bench_n2.json 2> gpurun_out/r5as_bench_n2.err || { tail -20 gpurun_out/r5as_bench_n2.err; exit 1; }
