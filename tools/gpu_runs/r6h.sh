# the local passes of a 1-rank, 4-pointer halving-doubling under rocprof
set -o pipefail
mkdir -p gpurun_out/r6h
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=$(mktemp -d)
bash tools/gpu_session.sh \
 "150:r6h_prof:rocprofv3 --kernel-trace --stats -d gpurun_out/r6h/prof -o mp -- python3 tools/multi_pointer_cost.py 0 1 $d 16777216 4 20"
