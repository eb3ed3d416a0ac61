#!/bin/bash
# r6d: RBN kernel + network tests (vs fp32), step-kernel audit (native axpy / fills), smoke score, db bench, profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q -s --timeout 250 --timeout-method thread tests/test_gpu_res_bn_fusion.py > gpurun_out/r6d_rbn_tests.log 2>&1; echo "rbn rc=$?"; grep -E "score|cos|passed|failed|Error" gpurun_out/r6d_rbn_tests.log | head -30
timeout -k 10 300 python3 -u -m pytest -x -q -s --timeout 250 --timeout-method thread tests/test_gpu_step_kernels.py > gpurun_out/r6d_step_kernels.log 2>&1; echo "step-kernels rc=$?"; grep -E "torch:|kernels,|passed|failed" gpurun_out/r6d_step_kernels.log | head -30
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6d_smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/r6d_smoke.log
timeout -k 10 300 python3 -u bench.py > gpurun_out/r6d_bench_db.log 2>&1 || { tail -20 gpurun_out/r6d_bench_db.log; exit 1; }
tail -1 gpurun_out/r6d_bench_db.log | cut -c1-200
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6d_prof" -o run -- python3 "$R/bench.py" --steps 8 --warmup 3 > "$R/gpurun_out/r6d_prof.log" 2>&1 || { tail -20 "$R/gpurun_out/r6d_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_summary.py $(ls gpurun_out/r6d_prof/*/run_results.db gpurun_out/r6d_prof/run_results.db 2>/dev/null | head -1) --steps 8 --top 40 > gpurun_out/r6d_prof_summary.txt 2>&1; head -50 gpurun_out/r6d_prof_summary.txt
