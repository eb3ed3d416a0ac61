#!/bin/bash
# Kernel-trace profile of the ResNet-50 bench (A/B via env passed by the caller); out dir $1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${1:-prof_resnet}
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$OUT" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 8 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/$OUT.log" 2>&1
rc=$?
grep -q '"metric"' "$GRAFT_REPO_ROOT/gpurun_out/$OUT.log" && echo "PROF_OK $OUT" || { echo "PROF_FAIL $OUT rc=$rc"; exit 1; }
