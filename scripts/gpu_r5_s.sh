#!/bin/bash
# r5: CU-masked side stream: external unmasked stream control + one profiled step at 192 CUs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
DL4J_AMD_WRW_CUS=256 timeout -k 10 200 python3 bench.py --steps 15 --warmup 4 > gpurun_out/r5s_zoo_256.log 2>&1 || { tail -5 gpurun_out/r5s_zoo_256.log; exit 1; }
echo "zoo cus=256(external) $(tail -1 gpurun_out/r5s_zoo_256.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
export DL4J_AMD_WRW_CUS=192
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r5s_prof" -o run -- python3 "$R/bench.py" --steps 3 --warmup 3 > "$R/gpurun_out/r5s_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r5s_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r5s_prof/run_results.db --top 30 > gpurun_out/r5s_step.txt && python3 tools/prof_steplist.py gpurun_out/r5s_prof/run_results.db > gpurun_out/r5s_steplist.txt && rm -rf gpurun_out/r5s_prof && head -12 gpurun_out/r5s_step.txt
