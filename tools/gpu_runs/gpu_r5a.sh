set -o pipefail
mkdir -p gpurun_out
timeout -k 10 90 tools/vmm_probe 1 > gpurun_out/r5a_vmm_1gib.jsonl 2> gpurun_out/r5a_vmm_1gib.err
rc=$?; echo "vmm 1 GiB rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 120 tools/vmm_probe 2.5 > gpurun_out/r5a_vmm_2p5gib.jsonl 2> gpurun_out/r5a_vmm_2p5gib.err
rc=$?; echo "vmm 2.5 GiB rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=0 -p no:cacheprovider --junitxml=gpurun_out/r5a_junit.xml > gpurun_out/r5a_pytest.log 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/r5a_pytest.log
