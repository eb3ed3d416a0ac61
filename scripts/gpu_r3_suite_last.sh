#!/bin/bash
# Whole GPU suite + smoke on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 480 python3 -u -m pytest tests -x -q -m gpu -rs --timeout 120 --timeout-method thread > gpurun_out/r3c_suite_last.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r3c_suite_last.log | head -30; tail -5 gpurun_out/r3c_suite_last.log; exit 1; }
tail -4 gpurun_out/r3c_suite_last.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c_smoke_last.log 2>&1 || { tail -20 gpurun_out/r3c_smoke_last.log; exit 1; }
tail -2 gpurun_out/r3c_smoke_last.log
