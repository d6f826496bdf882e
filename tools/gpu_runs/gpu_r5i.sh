set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/vmm_leak.py 40 > gpurun_out/r5i_vmm_leak.jsonl 2> gpurun_out/r5i_vmm_leak.err
rc=$?; echo "vmm rc=$rc"; [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
timeout -k 10 200 python tools/vmm_leak.py 40 GLOO_AMD_VMM_FREE_VA=1 > gpurun_out/r5i_vmm_freeva_leak.jsonl 2> gpurun_out/r5i_vmm_freeva_leak.err
echo "vmm free-va rc=$?"
