#!/bin/bash
# r5: canonical ResNet-50 (stride-1 stage 2, global average pool) at batch 512: throughput + one-step kernel table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --variant canonical --batch 512 --steps 20 --warmup 5 > gpurun_out/r5m_canon.log 2>&1 || { tail -20 gpurun_out/r5m_canon.log; exit 1; }
tail -1 gpurun_out/r5m_canon.log | cut -c1-200
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/r5m_prof" -o run -- python3 "$R/bench.py" --variant canonical --batch 512 --steps 3 --warmup 4 > "$R/gpurun_out/r5m_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r5m_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r5m_prof/run_results.db --top 40 > gpurun_out/r5m_canon_step.txt && python3 tools/prof_steplist.py gpurun_out/r5m_prof/run_results.db > gpurun_out/r5m_canon_steplist.txt && rm -rf gpurun_out/r5m_prof && head -44 gpurun_out/r5m_canon_step.txt
