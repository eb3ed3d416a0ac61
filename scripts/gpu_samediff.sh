#!/bin/bash
# SameDiff own-autodiff on the GPU: numerics tests, then the SameDiff LSTM and BERT benches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_samediff.py tests/test_gpu_lstm.py > gpurun_out/sd_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_samediff_lstm.py --steps 20 --warmup 3 > gpurun_out/sd_lstm.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_bert_samediff.py > gpurun_out/sd_bert.log 2>&1
rc=$?
tail -5 gpurun_out/sd_tests.log; cat gpurun_out/sd_lstm.log | tail -3; tail -3 gpurun_out/sd_bert.log
exit $rc
