#!/bin/bash
# r6s: fp32 path: GEMM tile/split probe, numerics, LeNet audit + bench + step list
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/f32_gemm_probe.py > gpurun_out/r6s_f32probe.txt 2>&1 || { tail -5 gpurun_out/r6s_f32probe.txt; exit 1; }
grep -v Warn gpurun_out/r6s_f32probe.txt
timeout -k 10 300 python3 -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_nd4j_ops.py tests/test_gpu_fallback.py tests/test_gpu_kernels.py tests/test_gpu_step_kernels.py > gpurun_out/r6s_tests.log 2>&1; rc=$?; grep -E "kernels,|torch:|passed|failed" gpurun_out/r6s_tests.log | tail -12; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r6s_tests.log | head -20; exit 1; }
timeout -k 10 200 python3 tools/bench_lenet.py --device cuda --graph 0 --steps 50 --warmup 5 > gpurun_out/r6s_lenet_eager.json 2>gpurun_out/r6s_lenet.err && timeout -k 10 200 python3 tools/bench_lenet.py --device cuda --graph 1 --steps 50 --warmup 5 > gpurun_out/r6s_lenet_graph.json 2>>gpurun_out/r6s_lenet.err || { tail -5 gpurun_out/r6s_lenet.err; exit 1; }
cat gpurun_out/r6s_lenet_eager.json gpurun_out/r6s_lenet_graph.json
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/gpurun_out/r6s_prof" -o run -- python3 "$R/tools/bench_lenet.py" --device cuda --graph 0 --steps 5 --warmup 3 > "$R/gpurun_out/r6s_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r6s_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_steplist.py gpurun_out/r6s_prof/run_results.db > gpurun_out/r6s_steplist.txt && rm -rf gpurun_out/r6s_prof && tail -3 gpurun_out/r6s_steplist.txt
