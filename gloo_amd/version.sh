#!/bin/sh
# Writes build/version.cc to stdout (see srchash.py).
exec python3 "$(dirname "$0")/srchash.py"
