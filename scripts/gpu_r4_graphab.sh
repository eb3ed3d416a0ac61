#!/bin/bash
# Eager vs HIP-graph replay of the ResNet-50 step, with and without the weight-gradient overlap stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { # tag env... -- args
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 $BARGS > gpurun_out/r4_gab_$tag.log 2>&1 || { tail -5 gpurun_out/r4_gab_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/r4_gab_$tag.log | cut -c80-140)"
}
BARGS="--graph 0" run eager_ws1 DL4J_AMD_WRW_STREAM=1
BARGS="--graph 0" run eager_ws0 DL4J_AMD_WRW_STREAM=0
BARGS="--graph 1" run graph_ws1 DL4J_AMD_WRW_STREAM=1
BARGS="--graph 1" run graph_ws0 DL4J_AMD_WRW_STREAM=0
BARGS="--graph 0" run eager_ws1b DL4J_AMD_WRW_STREAM=1
BARGS="--graph 0 --variant canonical" run canon_eager DL4J_AMD_WRW_STREAM=1
BARGS="--graph 1 --variant canonical" run canon_graph DL4J_AMD_WRW_STREAM=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_coop_guard.py tests/test_gpu_self_attention.py tests/test_gpu_transformer.py tests/test_gpu_lstm.py tests/test_gpu_lstm_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gab_tests.log 2>&1 || { tail -30 gpurun_out/r4_gab_tests.log; exit 1; }
tail -1 gpurun_out/r4_gab_tests.log
R=$(pwd); export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4_gab_prof" -o run -- python3 "$R/bench.py" --steps 4 --warmup 3 --graph 0 > "$R/gpurun_out/r4_gab_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r4_gab_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r4_gab_prof/run_results.db --top 45 > gpurun_out/r4_gab_step_eager.txt && python3 tools/prof_steplist.py gpurun_out/r4_gab_prof/run_results.db > gpurun_out/r4_gab_steplist_eager.txt && rm -rf gpurun_out/r4_gab_prof && head -30 gpurun_out/r4_gab_step_eager.txt
