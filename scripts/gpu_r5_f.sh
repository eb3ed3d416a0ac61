#!/bin/bash
# r5: epilogue diagnostics (no global stores / stores only) + ResNet numerics tests + bench memory report
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in nostore storeonly; do
  for s in "4096 2304 768" "4096 768 3072"; do
    echo "== $v" >> gpurun_out/r5f_stamps.log
    timeout -k 5 60 ./tools/native/gemm_stamps_$v $s 4 >> gpurun_out/r5f_stamps.log 2>&1 || exit 1
  done
done
cat gpurun_out/r5f_stamps.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_resnet_numerics.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r5f_num.log 2>&1; rc=$?
grep -E "score|cos|PASS|FAIL|Error|passed|failed" gpurun_out/r5f_num.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/r5f_bench.log 2>&1 || { tail -20 gpurun_out/r5f_bench.log; exit 1; }
tail -1 gpurun_out/r5f_bench.log
