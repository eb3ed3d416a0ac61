#!/bin/bash
# LSTM path on the GPU: kernel numerics tests, char-LM bench (sequence kernels vs per-step path), kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lstm.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_lstm.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/pytest_lstm.log; exit 1; }
tail -3 gpurun_out/pytest_lstm.log
timeout -k 10 300 python tools/bench_lstm.py --steps 5 --warmup 2 > gpurun_out/bench_lstm.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_lstm.log; exit 1; }
tail -1 gpurun_out/bench_lstm.log
DL4J_AMD_LSTM_COOP=0 timeout -k 10 300 python tools/bench_lstm.py --steps 5 --warmup 2 > gpurun_out/bench_lstm_nocoop.log 2>&1 || { echo BENCH2_FAIL; tail -30 gpurun_out/bench_lstm_nocoop.log; exit 1; }
tail -1 gpurun_out/bench_lstm_nocoop.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_lstm" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_lstm.py" --steps 2 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_lstm.log" 2>&1 || { echo PROF_FAIL; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_lstm.log"; exit 1; }
echo PROF_OK
