#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv_v3.py -k "halo" -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_tests_halo.log 2>&1 || { tail -40 gpurun_out/r3_tests_halo.log; exit 1; }
tail -2 gpurun_out/r3_tests_halo.log
timeout -k 10 120 python3 tools/wrw_halo_probe.py --variant 1 --splits 256 2>&1 | grep -v amdgpu
timeout -k 10 120 python3 tools/wrw_halo_probe.py --variant 1 --splits 128 2>&1 | grep -v amdgpu
timeout -k 10 400 python3 tools/wrw_halo_bench.py --batch 512 --reps 10 > gpurun_out/r3_wrw_halo_bench.log 2>&1 || { tail -20 gpurun_out/r3_wrw_halo_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3_wrw_halo_bench.log
