#!/bin/bash
# Tiled weight relayout: conv GPU tests, ResNet-50 bench (eager, bs512), one-step kernel table, per-shape conv table
# vs MIOpen at bs512.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_v3.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r4_conv_tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r4_conv_tests.log | head -30; tail -30 gpurun_out/r4_conv_tests.log; exit 1; }
tail -2 gpurun_out/r4_conv_tests.log
timeout -k 10 400 python3 bench.py --steps 30 --warmup 5 > gpurun_out/r4_conv_bench.log 2>&1 || { tail -20 gpurun_out/r4_conv_bench.log; exit 1; }
echo "resnet: $(tail -1 gpurun_out/r4_conv_bench.log | cut -c1-200)"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4_conv_prof" -o run -- python3 "$R/bench.py" --steps 4 --warmup 3 > "$R/gpurun_out/r4_conv_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r4_conv_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r4_conv_prof/run_results.db --top 45 > gpurun_out/r4_conv_step.txt && python3 tools/prof_steplist.py gpurun_out/r4_conv_prof/run_results.db > gpurun_out/r4_conv_steplist.txt && rm -rf gpurun_out/r4_conv_prof && head -24 gpurun_out/r4_conv_step.txt
timeout -k 10 600 python3 -u tools/conv_bench.py --batch 512 --reps 10 > gpurun_out/r4_conv_shapes.log 2>&1 || { tail -20 gpurun_out/r4_conv_shapes.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_conv_shapes.log | head -60
