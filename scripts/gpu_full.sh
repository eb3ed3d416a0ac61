#!/bin/bash
# Full GPU test suite (as the driver runs it) + smoke()
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_full.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_full.log; [ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" gpurun_out/gpu_full.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke.log 2>&1; tail -2 gpurun_out/smoke.log
