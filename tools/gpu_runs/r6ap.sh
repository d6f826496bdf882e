# the last tree of round 6: the whole GPU suite as the driver runs it, and smoke
set -o pipefail
bash tools/gpu_session.sh \
 "900:r6ap_pytest_gpu_all:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
 "200:r6ap_smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")'"
