#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
: timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bn_conv_tests.log 2>&1 || { tail -30 gpurun_out/bn_conv_tests.log; exit 1; }
:
timeout -k 10 300 python -u tools/wrw_ab.py --batch 512 > gpurun_out/wrw_ab.log 2>&1 || { tail -20 gpurun_out/wrw_ab.log; exit 1; }
tail -3 gpurun_out/wrw_ab.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_remap.log 2>&1 || { tail -20 gpurun_out/bench_remap.log; exit 1; }
tail -1 gpurun_out/bench_remap.log
bash scripts/prof_resnet.sh prof_resnet_ab
