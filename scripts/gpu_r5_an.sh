#!/bin/bash
# r5: GPU suite + smoke after the masking / dropout / loss-layer fixes, then three headline bench runs (run-to-run
# spread) and the bs512 point
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
j() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5an_suite.log 2>&1 || { tail -60 gpurun_out/r5an_suite.log; exit 1; }
tail -2 gpurun_out/r5an_suite.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5an_smoke.log 2>&1 || { tail -20 gpurun_out/r5an_smoke.log; exit 1; }
tail -1 gpurun_out/r5an_smoke.log
for r in 1; do
  timeout -k 10 200 python3 bench.py > gpurun_out/r5an_bench$r.log 2>&1 || { tail -5 gpurun_out/r5an_bench$r.log; exit 1; }
  echo "bs1024 run$r $(j gpurun_out/r5an_bench$r.log)"
done
timeout -k 10 200 python3 bench.py --batch 512 > gpurun_out/r5an_bench512.log 2>&1 || { tail -5 gpurun_out/r5an_bench512.log; exit 1; }
echo "bs512 $(j gpurun_out/r5an_bench512.log)"
