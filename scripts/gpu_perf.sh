#!/bin/bash
# Perf iteration: conv GPU tests, probes, bench (graph), kernel-trace profile. Every GPU step has its own time
# limit and the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_gpu_conv.py tests/test_gpu_kernels.py tests/test_gpu_stats.py -x -q > gpurun_out/pytest_perf.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/pytest_perf.log; exit 1; }
tail -2 gpurun_out/pytest_perf.log
if [ -n "$PROBE" ]; then
  timeout -k 10 300 python $PROBE > gpurun_out/probe.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/probe.log; exit 1; }
  cat gpurun_out/probe.log
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
echo PROF_OK
