#!/bin/bash
# SameDiff benches (LSTM char-LM, BERT import) + kernel-trace profile of the BERT one
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd "$R" && timeout -k 10 200 python -u tools/bench_samediff_lstm.py --steps 30 --warmup 3 > gpurun_out/sd_lstm.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_sd_bert" -o run -- python3 "$R/tools/bench_bert_samediff.py" --steps 5 --warmup 3 > "$R/gpurun_out/prof_sd_bert.log" 2>&1
grep -q '"metric"' "$R/gpurun_out/prof_sd_bert.log" && echo PROF_OK || { echo PROF_FAIL; exit 1; }
tail -1 "$R/gpurun_out/sd_lstm.log"
