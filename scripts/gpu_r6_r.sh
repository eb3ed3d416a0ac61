#!/bin/bash
# r6r: LeNet fp32 eager step, ordered dispatch list with grids
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && DL4J_AMD_GEMM_VERBOSE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/gpurun_out/r6r_prof" -o run -- python3 "$R/tools/bench_lenet.py" --device cuda --graph 0 --steps 5 --warmup 3 > "$R/gpurun_out/r6r_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r6r_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_steplist.py gpurun_out/r6r_prof/run_results.db > gpurun_out/r6r_steplist.txt && rm -rf gpurun_out/r6r_prof && cat gpurun_out/r6r_steplist.txt
