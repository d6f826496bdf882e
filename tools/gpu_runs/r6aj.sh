# config-4 sweep (1 KiB .. 256 MiB per rank, 4 rank threads on the one GPU): halving-doubling against AllreduceBcube
# (base 2 and base 4), default routes, interleaved by algorithm
set -o pipefail
mkdir -p gpurun_out/r6aj
bash tools/gpu_session.sh \
 "300:r6aj_hd:python -u tools/bench_collectives.py --ranks 4 --configs 4 --max-lg 28 --iters 20 > gpurun_out/r6aj/config4_hd_p4.jsonl" \
 "300:r6aj_b2:python -u tools/bench_collectives.py --ranks 4 --configs 4 --max-lg 28 --iters 20 --algo4 bcube --base 2 > gpurun_out/r6aj/config4_bcube_b2_p4.jsonl" \
 "300:r6aj_b4:python -u tools/bench_collectives.py --ranks 4 --configs 4 --max-lg 28 --iters 20 --algo4 bcube --base 4 > gpurun_out/r6aj/config4_bcube_b4_p4.jsonl" \
 "300:r6aj_b2ref:GLOO_AMD_MESH=0 python -u tools/bench_collectives.py --ranks 4 --configs 4 --max-lg 28 --iters 20 --algo4 bcube --base 2 > gpurun_out/r6aj/config4_bcube_b2_p4_mesh0.jsonl"
