# round-6 streaming levers, re-recorded (the first records, r6ad / r6ae, were lost to the next call's clean-up):
# the stripped 2R + 1W kernel with an LDS occupancy cap, XCD-contiguous tiles and wave-contiguous packets, and the
# product kernel's load order x occupancy cap at 16, 64 and 256 MiB per operand
set -o pipefail
mkdir -p gpurun_out/r6ag
bash tools/gpu_session.sh \
 "200:r6ag_levers:python -u tools/tune/hbm_ceiling.py --lib libceiling_pre.so --steps 500 --reps 5 --only R2W1_x,product_reduce_inplace > gpurun_out/r6ag/levers_64mib.jsonl" \
 "200:r6ag_16:python -u tools/tune/hbm_ceiling.py --lib libceiling_pre.so --mib 16 --steps 1000 --reps 6 --only product_reduce_inplace > gpurun_out/r6ag/product_16mib.jsonl" \
 "200:r6ag_256:python -u tools/tune/hbm_ceiling.py --lib libceiling_pre.so --mib 256 --steps 200 --reps 6 --only product_reduce_inplace > gpurun_out/r6ag/product_256mib.jsonl"
