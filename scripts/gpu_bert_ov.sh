#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_transformer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bert.log 2>&1 || { tail -40 gpurun_out/pytest_bert.log; exit 1; }
tail -1 gpurun_out/pytest_bert.log
DL4J_AMD_SIDE_GEMM=0 timeout -k 10 300 python tools/bench_bert.py --impl dl4j > gpurun_out/bench_bert_noov.log 2>&1 || { tail -30 gpurun_out/bench_bert_noov.log; exit 1; }
tail -1 gpurun_out/bench_bert_noov.log | cut -c1-200
timeout -k 10 300 python tools/bench_bert.py --impl dl4j > gpurun_out/bench_bert_ov.log 2>&1 || { tail -30 gpurun_out/bench_bert_ov.log; exit 1; }
tail -1 gpurun_out/bench_bert_ov.log | cut -c1-200
