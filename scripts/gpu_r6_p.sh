#!/bin/bash
# r6p: LeNet fp32 eager step: bench + one-step kernel table (in-tree kernels only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python3 tools/bench_lenet.py --device cuda --graph 0 --steps 50 --warmup 5 > gpurun_out/r6p_lenet_eager.json 2>gpurun_out/r6p_lenet.err || { tail -5 gpurun_out/r6p_lenet.err; exit 1; }
timeout -k 10 200 python3 tools/bench_lenet.py --device cuda --graph 1 --steps 50 --warmup 5 > gpurun_out/r6p_lenet_graph.json 2>>gpurun_out/r6p_lenet.err || { tail -5 gpurun_out/r6p_lenet.err; exit 1; }
cat gpurun_out/r6p_lenet_eager.json gpurun_out/r6p_lenet_graph.json
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/gpurun_out/r6p_prof" -o run -- python3 "$R/tools/bench_lenet.py" --device cuda --graph 0 --steps 5 --warmup 3 > "$R/gpurun_out/r6p_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r6p_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r6p_prof/run_results.db --top 30 > gpurun_out/r6p_step.txt && rm -rf gpurun_out/r6p_prof && cat gpurun_out/r6p_step.txt
