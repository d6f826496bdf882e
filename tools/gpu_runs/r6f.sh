# N=2 bench rehearsal on the cut tree, mid-size launches under rocprof, multi-pointer cost
set -o pipefail
mkdir -p gpurun_out/r6f
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_session.sh \
 "150:r6f_midprof:rocprofv3 --kernel-trace --stats -d gpurun_out/r6f/midprof -o mid -- python3 tools/midsize_chunks.py 14 20" \
 "200:r6f_mp2:bash tools/multi_pointer_cost.sh 2 16777216 4 20 > gpurun_out/r6f/multi_pointer_p2.jsonl" \
 "200:r6f_mp4:bash tools/multi_pointer_cost.sh 4 4194304 4 20 > gpurun_out/r6f/multi_pointer_p4.jsonl" \
 "600:r6f_bench2:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/r6f/bench_n2_one_gpu.json"
