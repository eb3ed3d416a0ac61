#!/bin/bash
# r6ze: final-tree validation: full GPU suite, smoke(), headline bench x2, and a rocprofv3 kernel-stats pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6ze_gpu_suite.log 2>&1; rc=$?; tail -2 gpurun_out/r6ze_gpu_suite.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r6ze_gpu_suite.log | head -20; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6ze_smoke.log 2>&1 || { tail -20 gpurun_out/r6ze_smoke.log; exit 1; }
tail -2 gpurun_out/r6ze_smoke.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6ze_bench_$i.json 2> gpurun_out/r6ze_bench_$i.err || { tail -5 gpurun_out/r6ze_bench_$i.err; exit 1; }
  cat gpurun_out/r6ze_bench_$i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6ze_prof -o r6ze -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/r6ze_prof.log 2>&1 || { tail -20 gpurun_out/r6ze_prof.log; exit 1; }
echo prof-ok
