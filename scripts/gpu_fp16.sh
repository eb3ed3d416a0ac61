#!/bin/bash
# fp16 transformer path + SameDiff tests, then BERT benches (CG bf16/fp16, SameDiff bf16)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_transformer.py \
  tests/test_gpu_samediff.py tests/test_gpu_nn_misc.py > gpurun_out/fp16_tests.log 2>&1
rc=$?
tail -4 gpurun_out/fp16_tests.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" gpurun_out/fp16_tests.log | head -30; exit $rc; }
timeout -k 10 200 python -u tools/bench_bert.py --steps 20 --warmup 4 --dtype fp16 > gpurun_out/bert_fp16.log 2>&1 && tail -1 gpurun_out/bert_fp16.log &&
timeout -k 10 200 python -u tools/bench_bert.py --steps 20 --warmup 4 > gpurun_out/bert_bf16.log 2>&1 && tail -1 gpurun_out/bert_bf16.log &&
timeout -k 10 200 python -u tools/bench_bert_samediff.py --steps 20 --warmup 3 > gpurun_out/sd_bert.log 2>&1 && tail -1 gpurun_out/sd_bert.log
