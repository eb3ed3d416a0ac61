#!/bin/bash
# Round re-entry check: full GPU suite + smoke + default bench + kernel-trace profile of the bench
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
bash scripts/gpu_full.sh || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
bash scripts/prof_resnet.sh prof_resnet_verify
