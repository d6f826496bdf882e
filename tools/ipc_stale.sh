#!/bin/bash
# Runs tools/ipc_stale for every writer (two processes on GPU 0); JSON lines
# on stdout.  Build: hipcc --offload-arch=gfx950 -O2 tools/ipc_stale.hip -o tools/ipc_stale
set -o pipefail
for w in ${WRITERS:-none kernel memcpy graph-kernel graph-memcpy}; do
  d=$(mktemp -d)
  timeout -k 5 60 tools/ipc_stale 1 "$d" "$w" ${ITERS:-4} &
  exp=$!
  timeout -k 5 60 tools/ipc_stale 0 "$d" "$w" ${ITERS:-4}
  imp=$?
  wait $exp
  ex=$?
  echo "{\"writer\": \"$w\", \"importer_exit\": $imp, \"exporter_exit\": $ex}"
  rm -rf "$d"
  if [ $imp -gt 1 ] || [ $ex -ne 0 ]; then exit 1; fi
done
