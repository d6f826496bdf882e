# round 5, GPU call e: VMM pool, quick checks first
set -o pipefail
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 200 python -u -m pytest "tests/test_transport_gpu.py::test_transport_receive_buffer_of_2p5gib_across_processes" "tests/test_collectives_gpu.py::test_processes_ipc" tests/test_ipc_pool_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider --durations=0 > gpurun_out/r5e_pytest_a.log 2>&1
rc=$?; echo "pytest a rc=$rc"; tail -3 gpurun_out/r5e_pytest_a.log
