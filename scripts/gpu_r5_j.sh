#!/bin/bash
# r5: in-tree-only GEMM by default (library opt-in, counted), tiled split-K fp32 kernel, lean GELU/dGELU epilogues
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_fallback.py tests/test_gpu_transformer.py tests/test_gpu_abi.py tests/test_gpu_samediff.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5j_tests.log 2>&1 || { tail -40 gpurun_out/r5j_tests.log; exit 1; }
tail -2 gpurun_out/r5j_tests.log
timeout -k 10 300 python3 -u tools/gemm_bench.py --rounds 3 > gpurun_out/r5j_gemm.log 2>&1 || { tail -20 gpurun_out/r5j_gemm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5j_gemm.log
timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 > gpurun_out/r5j_bert.log 2>&1 || { tail -20 gpurun_out/r5j_bert.log; exit 1; }
echo "bert: $(tail -1 gpurun_out/r5j_bert.log | cut -c1-150)"
timeout -k 10 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3 > gpurun_out/r5j_bsd.log 2>&1 || { tail -20 gpurun_out/r5j_bsd.log; exit 1; }
echo "bert samediff: $(tail -1 gpurun_out/r5j_bsd.log | cut -c1-150)"
timeout -k 10 300 python3 tools/bench_lenet.py --device cuda > gpurun_out/r5j_lenet.log 2>&1 || { tail -20 gpurun_out/r5j_lenet.log; exit 1; }
echo "lenet: $(tail -1 gpurun_out/r5j_lenet.log | cut -c1-200)"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5j_bench.log 2>&1 || { tail -20 gpurun_out/r5j_bench.log; exit 1; }
echo "resnet: $(tail -1 gpurun_out/r5j_bench.log | cut -c1-150)"
