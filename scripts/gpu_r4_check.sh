#!/bin/bash
# Round-4 iteration loop: a GPU test subset ($TESTS, default the BN/conv kernel tests), the ResNet-50 bench, and the
# last-step kernel table of the bench under rocprofv3 --kernel-trace.  Usage: scripts/gpu_r4_check.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
TAG=${1:-chk}
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_gpu_conv_v3.py tests/test_gpu_kernels.py tests/test_gpu_bnpool.py tests/test_gpu_bn_bwd_epilogue.py"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 500 python3 -u -m pytest $TESTS -x -q -rs --timeout 120 --timeout-method thread > gpurun_out/r4_${TAG}_tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4_${TAG}_tests.log | head -30; tail -30 gpurun_out/r4_${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/r4_${TAG}_tests.log
fi
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/r4_${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/r4_${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/r4_${TAG}_bench.log | cut -c1-220
[ -n "$NOPROF" ] && exit 0
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4_${TAG}_prof" -o run -- python3 "$R/bench.py" --steps 4 --warmup 3 ${BENCH_ARGS} > "$R/gpurun_out/r4_${TAG}_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r4_${TAG}_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r4_${TAG}_prof/run_results.db --top 45 > gpurun_out/r4_${TAG}_step.txt && rm -rf gpurun_out/r4_${TAG}_prof && head -30 gpurun_out/r4_${TAG}_step.txt
