#!/bin/bash
# r6q: fp32 conv as single GEMMs: numerics, LeNet GPU tests, LeNet bench + step table + torch-op sites
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nd4j_ops.py tests/test_gpu_fallback.py tests/test_gpu_kernels.py tests/test_gpu_gemm.py > gpurun_out/r6q_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r6q_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/r6q_tests.log | head -20; exit 1; }
timeout -k 10 200 python3 tools/bench_lenet.py --device cuda --graph 0 --steps 50 --warmup 5 > gpurun_out/r6q_lenet_eager.json 2>gpurun_out/r6q_lenet.err || { tail -5 gpurun_out/r6q_lenet.err; exit 1; }
timeout -k 10 200 python3 tools/bench_lenet.py --device cuda --graph 1 --steps 50 --warmup 5 > gpurun_out/r6q_lenet_graph.json 2>>gpurun_out/r6q_lenet.err || { tail -5 gpurun_out/r6q_lenet.err; exit 1; }
cat gpurun_out/r6q_lenet_eager.json gpurun_out/r6q_lenet_graph.json
timeout -k 10 200 python3 tools/step_torch_ops.py lenet > gpurun_out/r6q_lenet_ops.txt 2>&1 || { tail -5 gpurun_out/r6q_lenet_ops.txt; exit 1; }
grep -v "Warn\|warn\|amdgpu.ids" gpurun_out/r6q_lenet_ops.txt
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/gpurun_out/r6q_prof" -o run -- python3 "$R/tools/bench_lenet.py" --device cuda --graph 0 --steps 5 --warmup 3 > "$R/gpurun_out/r6q_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r6q_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r6q_prof/run_results.db --top 30 > gpurun_out/r6q_step.txt && rm -rf gpurun_out/r6q_prof && cat gpurun_out/r6q_step.txt
