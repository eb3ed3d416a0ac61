#!/bin/bash
# BN-backward epilogue modes 0 / 1 / 2 on the ResNet-50 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_bn_bwd_epilogue.py -x -q -rs --timeout 120 --timeout-method thread > gpurun_out/r3c_bnb3_tests.log 2>&1 || { tail -40 gpurun_out/r3c_bnb3_tests.log; exit 1; }
tail -1 gpurun_out/r3c_bnb3_tests.log
for m in 0 1 2; do
  DL4J_AMD_BN_BWD_EPILOGUE=$m timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3c_bench_bnbmode$m.log 2>&1 || { tail -20 gpurun_out/r3c_bench_bnbmode$m.log; exit 1; }
  echo "mode $m: $(tail -1 gpurun_out/r3c_bench_bnbmode$m.log | cut -c1-160)"
done
