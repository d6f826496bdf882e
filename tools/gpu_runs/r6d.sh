set -o pipefail
mkdir -p gpurun_out/r6d
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_session.sh \
 "200:r6d_staged:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_staged_gpu.py tests/test_reduce_gpu.py" \
 "200:r6d_smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")'" \
 "300:r6d_bench:python -u bench.py > gpurun_out/r6d/bench_n1.json" \
 "120:r6d_dmabuf:./tools/dmabuf_probe 4096 1048576 67108864 > gpurun_out/r6d/dmabuf_probe.jsonl" \
 "200:r6d_midsize:python -u tools/midsize_chunks.py 14 20 > gpurun_out/r6d/midsize_chunks.jsonl" \
 "200:r6d_hostsmall:python -u tools/host_small_reduce.py 200 > gpurun_out/r6d/host_small_reduce.jsonl" \
 "400:r6d_prof:rocprofv3 --kernel-trace --stats -d gpurun_out/r6d/prof -o r6d -- python3 bench.py --no-cpu --no-host-staged > gpurun_out/r6d/bench_n1_under_rocprof.json"
