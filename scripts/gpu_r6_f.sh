#!/bin/bash
# r6f: serial (no side stream) kernel table of the zoo bs1024 step on the round-6 tree: clean per-kernel attribution
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
export DL4J_AMD_WRW_STREAM=0
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r6f_prof" -o run -- python3 "$R/bench.py" --steps 3 --warmup 3 > "$R/gpurun_out/r6f_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r6f_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r6f_prof/run_results.db --top 70 > gpurun_out/r6f_step.txt && rm -rf gpurun_out/r6f_prof && head -50 gpurun_out/r6f_step.txt
