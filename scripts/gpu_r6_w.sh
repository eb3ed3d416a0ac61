#!/bin/bash
# r6w: ordered dispatch list of one serial-stream ResNet-50 bs1024 step (kernel -> call-site mapping)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
export DL4J_AMD_WRW_STREAM=0
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r6w_prof" -o run -- python3 "$R/bench.py" --steps 3 --warmup 3 > "$R/gpurun_out/r6w_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r6w_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_steplist.py gpurun_out/r6w_prof/run_results.db > gpurun_out/r6w_steplist.txt && rm -rf gpurun_out/r6w_prof && grep -n "igemm_fwd" gpurun_out/r6w_steplist.txt | head -20
