# round 5, GPU call d: the VMM cross-process pool (executor arenas / mailboxes, transport landing slabs)
set -o pipefail
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python -u -m pytest tests/test_transport_gpu.py tests/test_ipc_pool_gpu.py "tests/test_collectives_gpu.py::test_processes_ipc" -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider --durations=0 > gpurun_out/r5d_pytest_a.log 2>&1
rc=$?; echo "pytest a rc=$rc"; tail -3 gpurun_out/r5d_pytest_a.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_bandwidth_gpu.py -k "2gib or config3_full or halving_doubling_bandwidth" -m gpu -q --timeout 580 --timeout-method thread -p no:cacheprovider --durations=0 > gpurun_out/r5d_pytest_b.log 2>&1
rc=$?; echo "pytest b rc=$rc"; tail -3 gpurun_out/r5d_pytest_b.log; fatal $rc && exit $rc
timeout -k 10 700 python -u -m pytest tests/test_collectives_gpu.py tests/test_gloo_transport.py tests/test_newstyle_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider --durations=0 > gpurun_out/r5d_pytest_c.log 2>&1
rc=$?; echo "pytest c rc=$rc"; tail -3 gpurun_out/r5d_pytest_c.log
