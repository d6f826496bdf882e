# round 5, GPU call f: VMM pool diagnosis (short timeouts, per-rank logs)
set -o pipefail
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
run() { timeout -k 10 80 python tools/vmm_diag.py "$@"; rc=$?; echo "$1 rc=$rc"; fatal $rc && exit $rc; return 0; }
run hd2 halving_doubling 2 100003
run hd2_memcpy halving_doubling 2 100003 GLOO_AMD_COPY=memcpy GLOO_AMD_INTERP=0
run rc4_ring ring_chunked 4 100003 GLOO_AMD_RING_MESH=0
run rc8_memcpy ring_chunked 8 4194304 GLOO_AMD_COPY=memcpy
echo done
