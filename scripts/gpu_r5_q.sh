#!/bin/bash
# r5: BERT one-step kernel table, in-tree GEMMs only (lean GELU / dGELU epilogues)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/r5q_bprof" -o run -- python3 "$R/tools/bench_bert.py" --steps 4 --warmup 3 > "$R/gpurun_out/r5q_bprof.log" 2>&1 || { tail -5 "$R/gpurun_out/r5q_bprof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r5q_bprof/run_results.db --top 30 > gpurun_out/r5q_bert_step.txt && python3 tools/prof_steplist.py gpurun_out/r5q_bprof/run_results.db > gpurun_out/r5q_bert_steplist.txt && rm -rf gpurun_out/r5q_bprof && head -34 gpurun_out/r5q_bert_step.txt
