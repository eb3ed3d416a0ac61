#!/bin/bash
# r5: lean GEMM epilogue — gemm tests, stamps, K-scan probe, gemm table (lean vs generic), ResNet + BERT benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_resnet_numerics.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r5g_tests.log 2>&1 || { tail -40 gpurun_out/r5g_tests.log; exit 1; }
grep -E "score|cos|worst|passed|failed" gpurun_out/r5g_tests.log
for s in "4096 2304 768" "4096 768 3072" "4096 4096 4096"; do
  timeout -k 5 60 ./tools/native/gemm_stamps $s 4 >> gpurun_out/r5g_stamps.log 2>&1 || exit 1
done
cat gpurun_out/r5g_stamps.log
timeout -k 10 300 python3 -u tools/gemm_probe.py --M 4096 --N 2304 --ks 64,768,3072 --cfgs 4,0,2,3,5 --outs bf16 > gpurun_out/r5g_probe.log 2>&1 || exit 1
DL4J_AMD_GEMM_LEAN=0 timeout -k 10 300 python3 -u tools/gemm_probe.py --M 4096 --N 2304 --ks 64,768,3072 --cfgs 4,0,2,3,5 --outs bf16 >> gpurun_out/r5g_probe.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5g_probe.log
timeout -k 10 300 python3 -u tools/gemm_bench.py --rounds 3 > gpurun_out/r5g_gemm.log 2>&1 || { tail -20 gpurun_out/r5g_gemm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5g_gemm.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5g_bench.log 2>&1 || { tail -20 gpurun_out/r5g_bench.log; exit 1; }
tail -1 gpurun_out/r5g_bench.log
timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 > gpurun_out/r5g_bert.log 2>&1 || { tail -20 gpurun_out/r5g_bert.log; exit 1; }
tail -1 gpurun_out/r5g_bert.log | cut -c1-300
