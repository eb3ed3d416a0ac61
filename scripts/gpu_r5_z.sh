#!/bin/bash
# r5: fast-erf GELU epilogues + size-based non-temporal stores: GEMM GPU tests, BERT / zoo / canonical benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
j() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_transformer.py tests/test_gpu_samediff.py > gpurun_out/r5z_tests.log 2>&1 || { tail -20 gpurun_out/r5z_tests.log; exit 1; }
tail -1 gpurun_out/r5z_tests.log
timeout -k 10 300 python3 tools/bench_bert.py > gpurun_out/r5z_bert.log 2>&1 || { tail -5 gpurun_out/r5z_bert.log; exit 1; }
echo "bert $(j gpurun_out/r5z_bert.log)"
timeout -k 10 200 python3 bench.py > gpurun_out/r5z_zoo.log 2>&1 || { tail -5 gpurun_out/r5z_zoo.log; exit 1; }
echo "zoo $(j gpurun_out/r5z_zoo.log)"
timeout -k 10 200 python3 bench.py --variant canonical --batch 512 --steps 15 --warmup 4 > gpurun_out/r5z_canon.log 2>&1 || { tail -5 gpurun_out/r5z_canon.log; exit 1; }
echo "canon $(j gpurun_out/r5z_canon.log)"
