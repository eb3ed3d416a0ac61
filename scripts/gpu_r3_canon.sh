#!/bin/bash
# Canonical ResNet-50 bench + BERT kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 400 python3 bench.py --variant canonical --steps 10 --warmup 4 > gpurun_out/r3_bench_canonical2.log 2>&1 || { tail -20 gpurun_out/r3_bench_canonical2.log; exit 1; }
tail -1 gpurun_out/r3_bench_canonical2.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3_prof_bert5" -o run -- python3 "$R/tools/bench_bert.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3_prof_bert5.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_prof_bert5.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r3_prof_bert5/run_results.db --top 30 > gpurun_out/r3_prof_bert5_step.txt && rm -f gpurun_out/r3_prof_bert5/run_results.db && head -24 gpurun_out/r3_prof_bert5_step.txt
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3_prof_canon" -o run -- python3 "$R/bench.py" --variant canonical --steps 4 --warmup 3 > "$R/gpurun_out/r3_prof_canon.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_prof_canon.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r3_prof_canon/run_results.db --top 40 > gpurun_out/r3_prof_canon_step.txt && rm -f gpurun_out/r3_prof_canon/run_results.db && head -30 gpurun_out/r3_prof_canon_step.txt
