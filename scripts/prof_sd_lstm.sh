#!/bin/bash
# Kernel-trace profile of the SameDiff LSTM char-LM bench; out dir gpurun_out/prof_sd_lstm
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_sd_lstm" -o run -- python3 "$R/tools/bench_samediff_lstm.py" --steps 10 --warmup 3 > "$R/gpurun_out/prof_sd_lstm.log" 2>&1
grep -q '"metric"' "$R/gpurun_out/prof_sd_lstm.log" && echo PROF_OK || { echo PROF_FAIL; exit 1; }
