#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_fallback.py tests/test_gpu_conv_benchscale.py > gpurun_out/resnet_tests.log 2>&1; rc=$?
tail -3 gpurun_out/resnet_tests.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" gpurun_out/resnet_tests.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_resnet" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/gpurun_out/prof_resnet.log" 2>&1
grep -q '"metric"' "$R/gpurun_out/prof_resnet.log" && echo PROF_OK
