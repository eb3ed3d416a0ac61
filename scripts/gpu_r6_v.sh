#!/bin/bash
# r6v: full GPU suite; LeNet fp32 eager/graph; ResNet-50 bench; BERT bench (after the fp32 / torch-op / stream changes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6v_gpu_suite.log 2>&1; rc=$?; tail -3 gpurun_out/r6v_gpu_suite.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r6v_gpu_suite.log | head -20; exit 1; }
timeout -k 10 200 python3 tools/bench_lenet.py --device cuda --graph 0 --steps 100 --warmup 5 > gpurun_out/r6v_lenet_eager.json 2>/dev/null && timeout -k 10 200 python3 tools/bench_lenet.py --device cuda --graph 1 --steps 100 --warmup 5 > gpurun_out/r6v_lenet_graph.json 2>/dev/null || exit 1
cat gpurun_out/r6v_lenet_eager.json gpurun_out/r6v_lenet_graph.json
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6v_bench.json 2> gpurun_out/r6v_bench.err || { tail -5 gpurun_out/r6v_bench.err; exit 1; }
cat gpurun_out/r6v_bench.json
timeout -k 10 300 python3 tools/bench_bert.py > gpurun_out/r6v_bert.json 2> gpurun_out/r6v_bert.err || { tail -5 gpurun_out/r6v_bert.err; exit 1; }
cat gpurun_out/r6v_bert.json
