#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --variant canonical > gpurun_out/bench_canonical.log 2>&1 || { tail -20 gpurun_out/bench_canonical.log; exit 1; }
tail -1 gpurun_out/bench_canonical.log | cut -c1-220
DL4J_AMD_WRW_STREAM=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --variant canonical > gpurun_out/bench_canonical_noov.log 2>&1 || { tail -20 gpurun_out/bench_canonical_noov.log; exit 1; }
tail -1 gpurun_out/bench_canonical_noov.log | cut -c1-220
