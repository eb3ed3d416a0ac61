#!/bin/bash
# r6zc: in-kernel weight-gradient slab reduction tree (csrc/conv_wrw.hip tree_reduce): numerics tests, then the
# zoo ResNet-50 bench with the separate reduce launch (DL4J_AMD_WRW_TREE=0) against fan-ins 8 / 4 / 16
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv_v3.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "halo or wrw" > gpurun_out/r6zc_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r6zc_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r6zc_tests.log | head -20; exit 1; }
for f in 0 8 4 16 0 8; do
  DL4J_AMD_WRW_TREE=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6zc_bench_$f.json 2> gpurun_out/r6zc_bench_$f.err || { tail -5 gpurun_out/r6zc_bench_$f.err; exit 1; }
  echo "fan $f: $(tail -1 gpurun_out/r6zc_bench_$f.json | cut -c1-120)"
done
