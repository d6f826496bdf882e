# round 5, GPU call q: the whole GPU suite on the VMM pool (every runtime), with durations
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1080 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider --durations=40 > gpurun_out/r5q_pytest_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -60 gpurun_out/r5q_pytest_all.log
exit $rc
