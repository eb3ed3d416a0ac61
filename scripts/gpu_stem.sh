#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnpool.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stem_tests.log 2>&1 || { tail -30 gpurun_out/stem_tests.log; exit 1; }
tail -1 gpurun_out/stem_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_stem.log 2>&1 || { tail -20 gpurun_out/bench_stem.log; exit 1; }
tail -1 gpurun_out/bench_stem.log | cut -c1-200
bash scripts/prof_resnet.sh prof_resnet_stem
