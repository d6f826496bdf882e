# round 5, GPU call aa: stress with 16 / 64 MiB cases (eager + graph mesh plans, plain-store copy-out / fold / REDUCE)
set -o pipefail
mkdir -p gpurun_out/r5aa_stress
STRESS_BIG=1 timeout -k 10 200 python tools/stress.py 4 90 21 > gpurun_out/r5aa_stress/p4_mesh_big.jsonl 2> gpurun_out/r5aa_stress/p4_mesh_big.err || { tail -20 gpurun_out/r5aa_stress/p4_mesh_big.err; cat gpurun_out/r5aa_stress/p4_mesh_big.jsonl; exit 1; }
STRESS_BIG=1 GLOO_AMD_MESH=0 timeout -k 10 150 python tools/stress.py 3 60 22 > gpurun_out/r5aa_stress/p3_reference_big.jsonl 2> gpurun_out/r5aa_stress/p3_reference_big.err || { tail -20 gpurun_out/r5aa_stress/p3_reference_big.err; cat gpurun_out/r5aa_stress/p3_reference_big.jsonl; exit 1; }
STRESS_BIG=1 timeout -k 10 150 python tools/stress.py 2 60 23 > gpurun_out/r5aa_stress/p2_mesh_big.jsonl 2> gpurun_out/r5aa_stress/p2_mesh_big.err || { tail -20 gpurun_out/r5aa_stress/p2_mesh_big.err; cat gpurun_out/r5aa_stress/p2_mesh_big.jsonl; exit 1; }
tail -n 2 gpurun_out/r5aa_stress/*.jsonl
