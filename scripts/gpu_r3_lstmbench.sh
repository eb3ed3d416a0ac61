#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/bench_lstm.py --steps 5 --warmup 2 --graph 0 > gpurun_out/r3_bench_lstm_eager.log 2>&1 || exit 1
tail -1 gpurun_out/r3_bench_lstm_eager.log
timeout -k 10 200 python3 tools/bench_lstm.py --steps 5 --warmup 2 --graph 1 > gpurun_out/r3_bench_lstm.log 2>&1 || exit 1
tail -1 gpurun_out/r3_bench_lstm.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r3_prof_lstm" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_lstm.py" --steps 3 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/r3_prof_lstm.log" 2>&1; echo "prof rc=$?"
