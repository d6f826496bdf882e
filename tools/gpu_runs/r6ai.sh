# the whole GPU suite once more on the final tree (another box), as the driver runs it
set -o pipefail
bash tools/gpu_session.sh \
 "900:r6ai_pytest_gpu_all:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
