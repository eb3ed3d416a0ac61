#!/bin/bash
# r5: full GPU suite + smoke + headline / secondary benches after the epilogue changes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
j() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ab_suite.log 2>&1 || { tail -60 gpurun_out/r5ab_suite.log; exit 1; }
tail -2 gpurun_out/r5ab_suite.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ab_smoke.log 2>&1 || { tail -20 gpurun_out/r5ab_smoke.log; exit 1; }
tail -1 gpurun_out/r5ab_smoke.log
timeout -k 10 200 python3 bench.py > gpurun_out/r5ab_bench.log 2>&1 || { tail -5 gpurun_out/r5ab_bench.log; exit 1; }
echo "zoo bs1024 $(j gpurun_out/r5ab_bench.log)"
timeout -k 10 200 python3 bench.py --batch 512 > gpurun_out/r5ab_bench512.log 2>&1 || { tail -5 gpurun_out/r5ab_bench512.log; exit 1; }
echo "zoo bs512 $(j gpurun_out/r5ab_bench512.log)"
timeout -k 10 300 python3 tools/bench_bert.py > gpurun_out/r5ab_bert.log 2>&1 || { tail -5 gpurun_out/r5ab_bert.log; exit 1; }
echo "bert $(j gpurun_out/r5ab_bert.log)"
timeout -k 10 300 python3 tools/bench_bert.py --dtype fp16 > gpurun_out/r5ab_bert16.log 2>&1 || { tail -5 gpurun_out/r5ab_bert16.log; exit 1; }
echo "bert fp16 $(j gpurun_out/r5ab_bert16.log)"
timeout -k 10 300 python3 tools/bench_bert_samediff.py > gpurun_out/r5ab_sdbert.log 2>&1 || { tail -5 gpurun_out/r5ab_sdbert.log; exit 1; }
echo "samediff bert $(j gpurun_out/r5ab_sdbert.log)"
