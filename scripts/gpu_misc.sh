#!/bin/bash
# nn_misc kernels + SameDiff GPU tests, then SameDiff bench/profile
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_nn_misc.py \
  > gpurun_out/misc_tests.log 2>&1
rc=$?
tail -25 gpurun_out/misc_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/prof_sd.sh
