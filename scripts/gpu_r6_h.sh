#!/bin/bash
# r6h: halo conv kernel iteration: numerics + per-shape bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_halo.py > gpurun_out/r6h_halo_tests.log 2>&1; rc=$?; echo "halo tests rc=$rc"; tail -5 gpurun_out/r6h_halo_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 tools/conv_stream_bench.py > gpurun_out/r6h_conv.log 2>&1 || { tail -20 gpurun_out/r6h_conv.log; exit 1; }
grep -E "shape|3,3\)" gpurun_out/r6h_conv.log
