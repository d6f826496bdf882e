# round 5, GPU call c: uncached VMM probe, inbox memory kinds, transport (fixed ticket zeroing) + rocprof,
# inconsistent-plan and pool-churn tests, copy engines on fine-grained sources
set -o pipefail
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 90 tools/vmm_probe 2.5 fresh uncached > gpurun_out/r5c_vmm_fresh_uncached.jsonl 2> gpurun_out/r5c_vmm_fresh_uncached.err
rc=$?; echo "vmm uncached rc=$rc"; fatal $rc && exit $rc
timeout -k 10 120 tools/mem_kinds_bw > gpurun_out/r5c_mem_kinds_bw.jsonl 2> gpurun_out/r5c_mem_kinds_bw.err
rc=$?; echo "mem kinds rc=$rc"; fatal $rc && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_transport_gpu.py tests/test_gloo_transport.py tests/test_ipc_pool_gpu.py "tests/test_collectives_gpu.py::test_rank_inconsistent_plan_is_refused" -m gpu -q --timeout 390 --timeout-method thread -p no:cacheprovider --durations=0 > gpurun_out/r5c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5c_pytest.log; fatal $rc && exit $rc
tools/transport_bench_prof.sh $PWD/gpurun_out/r5c_prof_tbench_device device > gpurun_out/r5c_prof_tbench_device.jsonl 2> gpurun_out/r5c_prof_tbench_device.err
rc=$?; echo "tbench prof rc=$rc"; fatal $rc && exit $rc
for m in coarse fine; do
  COPY_SRC_MEM=$m COPY_MIB=8,32 COPY_BLOCKS=256,1024 timeout -k 10 120 python tools/copy_engines.py > gpurun_out/r5c_copy_engines_src_$m.jsonl 2> gpurun_out/r5c_copy_engines_src_$m.err
  rc=$?; echo "copy engines $m rc=$rc"; fatal $rc && exit $rc
done
