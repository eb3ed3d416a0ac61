#!/bin/bash
# r6e: full GPU suite after the round-6 kernel changes, smoke (pinned band), db bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r6e_gpu_suite.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -15 gpurun_out/r6e_gpu_suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6e_smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r6e_smoke.log
