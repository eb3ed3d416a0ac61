#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u tools/conv_bench.py --batch 512 --reps 10 > gpurun_out/conv_bench512.log 2>&1 || { tail -20 gpurun_out/conv_bench512.log; exit 1; }
tail -25 gpurun_out/conv_bench512.log
