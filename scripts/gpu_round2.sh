#!/bin/bash
# Round-2 integration check: full GPU suite, ResNet-50 bench, BERT + LSTM benches, BERT kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 python tools/bench_bert.py --impl dl4j > gpurun_out/bench_bert.log 2>&1 || { echo BERT_FAIL; tail -30 gpurun_out/bench_bert.log; exit 1; }
tail -1 gpurun_out/bench_bert.log
timeout -k 10 300 python tools/bench_lstm.py --steps 5 --warmup 2 > gpurun_out/bench_lstm.log 2>&1 || { echo LSTM_FAIL; tail -30 gpurun_out/bench_lstm.log; exit 1; }
tail -1 gpurun_out/bench_lstm.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bert" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_bert.py" --steps 3 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof_bert.log" 2>&1 || { echo PROF_FAIL; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_bert.log"; exit 1; }
echo PROF_OK
