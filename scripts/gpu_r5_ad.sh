#!/bin/bash
# r5: kernel table of the in-process world-1 step (graphs + accumulator) to compare with the eager headline step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/r5ad_prof" -o run -- python3 "$R/bench.py" --gpus 1 --inprocess 1 --steps 3 --warmup 3 > "$R/gpurun_out/r5ad_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r5ad_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r5ad_prof/run_results.db --top 60 > gpurun_out/r5ad_step.txt && python3 tools/prof_steplist.py gpurun_out/r5ad_prof/run_results.db > gpurun_out/r5ad_steplist.txt && rm -rf gpurun_out/r5ad_prof && head -3 gpurun_out/r5ad_step.txt
