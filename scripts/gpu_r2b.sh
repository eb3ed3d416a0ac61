#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_bert.py --impl dl4j --warmup 4 > gpurun_out/bench_bert.log 2>&1 || { echo BERT_FAIL; tail -30 gpurun_out/bench_bert.log; exit 1; }
tail -1 gpurun_out/bench_bert.log
timeout -k 10 300 python tools/bench_bert.py --impl dl4j --graph 0 > gpurun_out/bench_bert_eager.log 2>&1 || { echo BERT2_FAIL; tail -30 gpurun_out/bench_bert_eager.log; exit 1; }
tail -1 gpurun_out/bench_bert_eager.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bert" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_bert.py" --steps 20 --warmup 4 > "$GRAFT_REPO_ROOT/gpurun_out/prof_bert.log" 2>&1 || { echo PROF_FAIL; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_bert.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_lstm" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_lstm.py" --steps 3 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof_lstm.log" 2>&1 || { echo PROF2_FAIL; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_lstm.log"; exit 1; }
echo PROF_OK
