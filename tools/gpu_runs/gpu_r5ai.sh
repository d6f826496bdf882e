# round 5, GPU call ai: 2-rank bench rehearsals, done signal on (default) vs off, interleaved
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export GLOO_AMD_DONE_SPIN=0; else unset GLOO_AMD_DONE_SPIN; fi
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2952$rep bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-host-staged > gpurun_out/r5ai_bench_n2_${v}_${rep}.json 2> gpurun_out/r5ai_bench_n2_${v}_${rep}.err || { tail -20 gpurun_out/r5ai_bench_n2_${v}_${rep}.err; exit 1; }
  done
done
