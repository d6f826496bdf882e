#!/bin/bash
# Runs tools/ipc_reuse in every mode (two processes on GPU 0); JSON lines on stdout.
set -o pipefail
for mode in ${MODES:-free-close pool-close pool-keep free-keep twobuf-close}; do
  d=$(mktemp -d)
  timeout -k 5 60 tools/ipc_reuse 1 "$d" "$mode" 6 &
  exp=$!
  timeout -k 5 60 tools/ipc_reuse 0 "$d" "$mode" 6
  imp=$?
  wait $exp
  ex=$?
  echo "{\"mode\": \"$mode\", \"importer_exit\": $imp, \"exporter_exit\": $ex}"
  rm -rf "$d"
  if [ $imp -gt 1 ] || [ $ex -ne 0 ]; then exit 1; fi
done
