#!/bin/bash
# Interleaved A/B of two libswarm builds on one box: election (tools/elect_ab.py) and allocation
# (tools/alloc_ab.py) at C3.  Usage: bash tools/ab_libs.sh LIB_A LIB_B [ROUNDS]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 "${3:-2}"); do
  for lib in "$1" "$2"; do
    timeout -k 10 200 python -u tools/elect_ab.py "$lib" || exit $?
    timeout -k 10 200 python -u tools/alloc_ab.py "$lib" || exit $?
  done
done
