#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_samediff.py tests/test_gpu_lstm.py > gpurun_out/sd_tests.log 2>&1; rc=$?
tail -3 gpurun_out/sd_tests.log; [ $rc -eq 0 ] || { grep -n "Error\|assert\|WARN" gpurun_out/sd_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/bench_bert_samediff.py --steps 20 --warmup 3 > gpurun_out/sd_bert.log 2>&1; tail -2 gpurun_out/sd_bert.log
timeout -k 10 300 python -u tools/bench_bert_samediff.py --steps 20 --warmup 3 --dtype fp16 > gpurun_out/sd_bert_fp16.log 2>&1; tail -2 gpurun_out/sd_bert_fp16.log
