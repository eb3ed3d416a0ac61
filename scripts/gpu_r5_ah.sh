#!/bin/bash
# r5: full GPU suite + smoke + headline bench after the masking / parameter semantics fixes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ah_suite.log 2>&1 || { tail -60 gpurun_out/r5ah_suite.log; exit 1; }
tail -2 gpurun_out/r5ah_suite.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ah_smoke.log 2>&1 || { tail -20 gpurun_out/r5ah_smoke.log; exit 1; }
tail -1 gpurun_out/r5ah_smoke.log
timeout -k 10 200 python3 bench.py > gpurun_out/r5ah_bench.log 2>&1 || { tail -5 gpurun_out/r5ah_bench.log; exit 1; }
tail -1 gpurun_out/r5ah_bench.log | cut -c1-200
