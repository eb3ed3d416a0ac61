#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3_prof_halo" -o run -- python3 "$R/tools/wrw_halo_bench.py" --batch 512 --reps 5 > "$R/gpurun_out/r3_prof_halo.log" 2>&1
echo "rc=$?"
