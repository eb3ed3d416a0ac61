#!/bin/bash
# Phase-split strided bwd-data: conv / deconv GPU tests, canonical bench, zoo step dispatch list with stream ids.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_nn_misc.py -x -v --timeout 120 --timeout-method thread -k "phase or fwd_bwd or accumulates or deconv or Deconv" > gpurun_out/r3_tests_phase.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3_tests_phase.log | head -30; tail -5 gpurun_out/r3_tests_phase.log; exit 1; }
tail -1 gpurun_out/r3_tests_phase.log
timeout -k 10 400 python3 bench.py --variant canonical --steps 10 --warmup 4 > gpurun_out/r3_bench_canonical_phase.log 2>&1 || { tail -20 gpurun_out/r3_bench_canonical_phase.log; exit 1; }
tail -1 gpurun_out/r3_bench_canonical_phase.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3_prof_zoo" -o run -- python3 "$R/bench.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3_prof_zoo.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_prof_zoo.log"; exit 1; }
cd "$R" && python3 tools/prof_steplist.py gpurun_out/r3_prof_zoo/run_results.db > gpurun_out/r3_zoo_steplist.txt && python3 tools/prof_laststep.py gpurun_out/r3_prof_zoo/run_results.db --top 40 > gpurun_out/r3_zoo_step.txt && rm -f gpurun_out/r3_prof_zoo/run_results.db && tail -1 gpurun_out/r3_zoo_steplist.txt && head -12 gpurun_out/r3_zoo_step.txt
