#!/bin/bash
# Full GPU test suite + smoke (what the driver runs at round end).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_gpu_full.log 2>&1; rc=$?
grep -E "FAIL|Error" gpurun_out/r3_gpu_full.log | head -20; tail -3 gpurun_out/r3_gpu_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1; rc=$?
tail -3 gpurun_out/r3_smoke.log; exit $rc
