#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$R/gpurun_out/prof_copies" -o run -- python3 "$R/bench.py" --steps 3 --warmup 2 --batch 128 > "$R/gpurun_out/prof_copies.log" 2>&1
grep -q '"metric"' "$R/gpurun_out/prof_copies.log" && echo PROF_OK
