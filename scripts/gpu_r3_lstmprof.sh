#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3_prof_lstm" -o run -- python3 "$R/tools/bench_lstm.py" --steps 3 --warmup 2 --graph 0 > "$R/gpurun_out/r3_prof_lstm.log" 2>&1; echo "prof rc=$?"
tail -1 "$R/gpurun_out/r3_prof_lstm.log"
