#!/bin/bash
# r5 final: full GPU suite + smoke + headline bench (defaults) + secondary benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
j() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("kernel_db", d.get("kernel_db")))'; }
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ag_suite.log 2>&1 || { tail -60 gpurun_out/r5ag_suite.log; exit 1; }
tail -2 gpurun_out/r5ag_suite.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ag_smoke.log 2>&1 || { tail -20 gpurun_out/r5ag_smoke.log; exit 1; }
tail -1 gpurun_out/r5ag_smoke.log
timeout -k 10 200 python3 bench.py > gpurun_out/r5ag_bench.log 2>&1 || { tail -5 gpurun_out/r5ag_bench.log; exit 1; }
echo "zoo bs1024 $(j gpurun_out/r5ag_bench.log)"
tail -1 gpurun_out/r5ag_bench.log
timeout -k 10 200 python3 bench.py --batch 512 > gpurun_out/r5ag_bench512.log 2>&1 || { tail -5 gpurun_out/r5ag_bench512.log; exit 1; }
echo "zoo bs512 $(j gpurun_out/r5ag_bench512.log)"
timeout -k 10 300 python3 tools/bench_lstm.py > gpurun_out/r5ag_lstm.log 2>&1 || { tail -5 gpurun_out/r5ag_lstm.log; exit 1; }
echo "lstm $(tail -1 gpurun_out/r5ag_lstm.log | cut -c1-160)"
timeout -k 10 300 python3 tools/bench_samediff_lstm.py > gpurun_out/r5ag_sdlstm.log 2>&1 || { tail -5 gpurun_out/r5ag_sdlstm.log; exit 1; }
echo "sdlstm $(tail -1 gpurun_out/r5ag_sdlstm.log | cut -c1-160)"
timeout -k 10 300 python3 tools/bench_lenet.py > gpurun_out/r5ag_lenet.log 2>&1 || { tail -5 gpurun_out/r5ag_lenet.log; exit 1; }
echo "lenet $(tail -1 gpurun_out/r5ag_lenet.log | cut -c1-160)"
