#!/bin/bash
# BN per-shape bench (+ kernel stats), fold reducers with batched loads; LN/BN tests; BERT + ResNet benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_transformer.py tests/test_gpu_conv.py -x -q --timeout 300 --timeout-method thread -k "batchnorm or layernorm or bn_stats" > gpurun_out/r3_tests_bn5.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3_tests_bn5.log | head -30; tail -5 gpurun_out/r3_tests_bn5.log; exit 1; }
tail -1 gpurun_out/r3_tests_bn5.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3_prof_bnbench" -o run -- python3 "$R/tools/bn_bench.py" > "$R/gpurun_out/r3_bn_bench.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_bn_bench.log"; exit 1; }
cd "$R" && grep -v "^W20\|^E20" gpurun_out/r3_bn_bench.log | tail -12
f=$(ls gpurun_out/r3_prof_bnbench/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print('%9.1f us %6s calls %8.2f us avg  %s' % (float(r['TotalDurationNs'])/1e3, r['Calls'], float(r['AverageNs'])/1e3, r['Name'][:90]))
" | tee gpurun_out/r3_bn_bench_kernels.txt
rm -f gpurun_out/r3_prof_bnbench/*.db
timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 > gpurun_out/r3_bench_bert5.log 2>&1 || { tail -20 gpurun_out/r3_bench_bert5.log; exit 1; }
tail -1 gpurun_out/r3_bench_bert5.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_bn5.log 2>&1 || { tail -20 gpurun_out/r3_bench_bn5.log; exit 1; }
tail -1 gpurun_out/r3_bench_bn5.log
