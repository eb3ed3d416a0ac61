#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lstm.py tests/test_gpu_fallback.py tests/test_gpu_gemm.py > gpurun_out/lstm_tests.log 2>&1; rc=$?
tail -3 gpurun_out/lstm_tests.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" gpurun_out/lstm_tests.log | head; exit $rc; }
timeout -k 10 300 python -u tools/bench_lstm.py --steps 3 --warmup 1 > gpurun_out/bench_lstm.log 2>&1 && tail -1 gpurun_out/bench_lstm.log &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_lstm" -o run -- python3 "$R/tools/bench_lstm.py" --steps 1 --warmup 1 > "$R/gpurun_out/prof_lstm.log" 2>&1
grep -q '"metric"' "$R/gpurun_out/prof_lstm.log" && echo PROF_OK
