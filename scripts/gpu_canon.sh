#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nn_misc.py > gpurun_out/misc_tests.log 2>&1; rc=$?
tail -3 gpurun_out/misc_tests.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" gpurun_out/misc_tests.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --variant canonical > gpurun_out/bench_canonical.log 2>&1 && tail -1 gpurun_out/bench_canonical.log
