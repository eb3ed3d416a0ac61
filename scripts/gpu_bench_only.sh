#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_only.log 2>&1 || { tail -20 gpurun_out/bench_only.log; exit 1; }
tail -1 gpurun_out/bench_only.log | cut -c1-200
timeout -k 10 300 python -u bench.py > gpurun_out/bench_only2.log 2>&1 || { tail -20 gpurun_out/bench_only2.log; exit 1; }
tail -1 gpurun_out/bench_only2.log | cut -c1-200
