#!/bin/bash
# r6j: halo conv with the epilogue overlapped: numerics, timing probe, per-shape bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_halo.py > gpurun_out/r6j_halo_tests.log 2>&1; rc=$?; echo "halo tests rc=$rc"; tail -5 gpurun_out/r6j_halo_tests.log
[ $rc -eq 0 ] || exit 1
for d in 0 1 2 3; do DL4J_AMD_HALO_DBG=$d timeout -k 10 120 python3 tools/halo_probe.py || exit 1; done
DL4J_AMD_HALO_DBG=0 timeout -k 10 120 python3 tools/halo_probe.py --hw 56 --batch 256 || exit 1
