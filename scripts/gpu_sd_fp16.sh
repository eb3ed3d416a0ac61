#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_bert_samediff.py --steps 20 --warmup 3 --dtype fp16 > gpurun_out/sd_bert_fp16.log 2>&1 && tail -1 gpurun_out/sd_bert_fp16.log &&
timeout -k 10 300 python -u tools/bench_bert_samediff.py --steps 20 --warmup 3 > gpurun_out/sd_bert.log 2>&1 && tail -1 gpurun_out/sd_bert.log
