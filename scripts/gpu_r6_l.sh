#!/bin/bash
# r6l: halo conv chosen for the 3x3 64->64 stage-2 convs (tunedb): bench, then a serial kernel table of the step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6l_bench.json 2> gpurun_out/r6l_bench.err || { tail -20 gpurun_out/r6l_bench.err; exit 1; }
cat gpurun_out/r6l_bench.json
export DL4J_AMD_WRW_STREAM=0
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r6l_prof" -o run -- python3 "$R/bench.py" --steps 3 --warmup 3 > "$R/gpurun_out/r6l_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r6l_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r6l_prof/run_results.db --top 70 > gpurun_out/r6l_step.txt && rm -rf gpurun_out/r6l_prof && head -40 gpurun_out/r6l_step.txt
