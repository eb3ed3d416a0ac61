#!/bin/bash
# r5: serial (no side stream) kernel table of the zoo bs1024 step: clean per-kernel attribution
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
export DL4J_AMD_WRW_STREAM=0
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r5u_prof" -o run -- python3 "$R/bench.py" --steps 3 --warmup 3 > "$R/gpurun_out/r5u_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r5u_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r5u_prof/run_results.db --top 60 > gpurun_out/r5u_step.txt && python3 tools/prof_steplist.py gpurun_out/r5u_prof/run_results.db > gpurun_out/r5u_steplist.txt && rm -rf gpurun_out/r5u_prof && head -3 gpurun_out/r5u_step.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r5u_cprof" -o run -- python3 "$R/bench.py" --variant canonical --batch 512 --steps 3 --warmup 3 > "$R/gpurun_out/r5u_cprof.log" 2>&1 || { tail -5 "$R/gpurun_out/r5u_cprof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r5u_cprof/run_results.db --top 60 > gpurun_out/r5u_cstep.txt && python3 tools/prof_steplist.py gpurun_out/r5u_cprof/run_results.db > gpurun_out/r5u_csteplist.txt && rm -rf gpurun_out/r5u_cprof && head -3 gpurun_out/r5u_cstep.txt
