#!/bin/bash
# Transformer path on the GPU: kernel + model numerics tests, BERT-base bench (ours vs PyTorch comparator), profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_transformer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bert.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/pytest_bert.log; exit 1; }
tail -2 gpurun_out/pytest_bert.log
timeout -k 10 300 python tools/bench_bert.py --impl dl4j > gpurun_out/bench_bert.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_bert.log; exit 1; }
tail -1 gpurun_out/bench_bert.log
timeout -k 10 300 python tools/bench_bert.py --impl torch > gpurun_out/bench_bert_torch.log 2>&1 || { echo BENCH2_FAIL; tail -30 gpurun_out/bench_bert_torch.log; exit 1; }
tail -1 gpurun_out/bench_bert_torch.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bert" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_bert.py" --steps 3 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof_bert.log" 2>&1 || { echo PROF_FAIL; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_bert.log"; exit 1; }
echo PROF_OK
