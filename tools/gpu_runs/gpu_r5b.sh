# round 5, GPU call b: VMM probe (fresh / same VA), transport tests + bench, batched suites
set -o pipefail
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for m in fresh; do  # "same" faulted the GPU once (r5b_vmm_same_va.err): never again
  timeout -k 10 90 tools/vmm_probe 2.5 $m > gpurun_out/r5b_vmm_$m.jsonl 2> gpurun_out/r5b_vmm_$m.err
  rc=$?; echo "vmm $m rc=$rc"; fatal $rc && exit $rc
done
timeout -k 10 400 python -u -m pytest tests/test_transport_gpu.py tests/test_gloo_transport.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5b_transport_pytest.log 2>&1
rc=$?; echo "transport pytest rc=$rc"; tail -3 gpurun_out/r5b_transport_pytest.log; fatal $rc && exit $rc
for kind in device host; do
  for pub in device hostfn; do
    if [ $pub = hostfn ]; then export GLOO_AMD_TRANSPORT_HOSTFN=1; else unset GLOO_AMD_TRANSPORT_HOSTFN; fi
    GLOO_BENCH_MIN_MS=200 BENCH_TIMEOUT=200 tools/transport_bench.sh $kind > gpurun_out/r5b_tbench_${kind}_${pub}.jsonl 2> gpurun_out/r5b_tbench_${kind}_${pub}.err
    rc=$?; echo "tbench $kind $pub rc=$rc"; fatal $rc && exit $rc
  done
done
unset GLOO_AMD_TRANSPORT_HOSTFN
timeout -k 10 900 python -u -m pytest tests/test_collectives_gpu.py tests/test_gloo_collectives.py tests/test_newstyle_gpu.py -m gpu -q --timeout 300 --timeout-method thread --durations=0 -p no:cacheprovider > gpurun_out/r5b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5b_pytest.log
