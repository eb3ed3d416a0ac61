#!/bin/bash
# Secondary benches on the final tree: canonical ResNet-50, BERT-base fp16, SameDiff BERT / LSTM.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 240 python3 bench.py --variant canonical --steps 10 --warmup 3 > gpurun_out/r3c_bench_canonical_final.log 2>&1 || { tail -20 gpurun_out/r3c_bench_canonical_final.log; exit 1; }
tail -1 gpurun_out/r3c_bench_canonical_final.log | cut -c1-160
timeout -k 10 240 python3 tools/bench_bert.py --dtype fp16 --steps 10 --warmup 3 > gpurun_out/r3c_bench_bert_fp16_final.log 2>&1 || { tail -20 gpurun_out/r3c_bench_bert_fp16_final.log; exit 1; }
tail -1 gpurun_out/r3c_bench_bert_fp16_final.log | cut -c1-160
timeout -k 10 240 python3 tools/bench_bert_samediff.py > gpurun_out/r3c_bench_bert_samediff_final.log 2>&1 || { tail -20 gpurun_out/r3c_bench_bert_samediff_final.log; exit 1; }
tail -1 gpurun_out/r3c_bench_bert_samediff_final.log | cut -c1-160
timeout -k 10 240 python3 tools/bench_samediff_lstm.py > gpurun_out/r3c_bench_samediff_lstm_final.log 2>&1 || { tail -20 gpurun_out/r3c_bench_samediff_lstm_final.log; exit 1; }
tail -1 gpurun_out/r3c_bench_samediff_lstm_final.log | cut -c1-160
