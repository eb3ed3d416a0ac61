#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/wrw_halo_bench.py --batch 512 --reps 10 > gpurun_out/r3_wrw_halo_bench.log 2>&1 || { tail -20 gpurun_out/r3_wrw_halo_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3_wrw_halo_bench.log
