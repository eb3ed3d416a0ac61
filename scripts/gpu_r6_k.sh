#!/bin/bash
# r6k: halo conv, 8 consumer waves: numerics + timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_halo.py > gpurun_out/r6k_halo_tests.log 2>&1; rc=$?; echo "halo tests rc=$rc"; tail -5 gpurun_out/r6k_halo_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python3 tools/halo_probe.py && timeout -k 10 120 python3 tools/halo_probe.py --hw 56 --batch 256
