#!/bin/bash
# Diagnosis of stale IPC imports: bench.py's config-3 variants
# in the order that provoked them, every arena export /
# import / close logged with probes of a failing mapping.
# usage (GPU box): bash tools/ipc_diag.sh TAG [REPEATS] [ORDER]
set -o pipefail
tag=${1:-diag}
reps=${2:-2}
order=${3:-ring_memcpy,ring_kernel,mesh_memcpy_forked,ring_kernel}
mkdir -p gpurun_out
for i in $(seq 1 "$reps"); do
  GLOO_AMD_IPC_DIAG=1 timeout -k 10 240 \
    python -u bench.py --gpus 2 --steps 5 --warmup 2 --config3-only --config3-variants "$order" \
    > gpurun_out/${tag}_$i.out 2> gpurun_out/${tag}_$i.err
  rc=$?
  echo "run $i rc $rc"
  grep -h "MISMATCH\|^{" gpurun_out/${tag}_$i.err gpurun_out/${tag}_$i.out | cut -c1-600 || true
  python3 - "$tag" "$i" <<'PY' || true
import json, sys
tag, i = sys.argv[1], sys.argv[2]
lines = [l for l in open(f"gpurun_out/{tag}_{i}.out") if l.startswith("{")]
if lines:
    x = json.loads(lines[-1]).get("xgmi_allreduce", {})
    print("default verified", x.get("verified"))
    for k, v in x.get("variants", {}).items():
        print(k, "verified", v.get("verified"), (v.get("error") or "")[:300])
PY
  [ $rc -eq 0 ] || exit $rc
done
