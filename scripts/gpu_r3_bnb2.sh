#!/bin/bash
# BN-backward epilogue incl. residual BNs: tests, bench A/B, one rocprof kernel trace (last-step table + dispatch list).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_bn_bwd_epilogue.py -x -q -rs --timeout 120 --timeout-method thread > gpurun_out/r3c_bnb2_tests.log 2>&1 || { tail -40 gpurun_out/r3c_bnb2_tests.log; exit 1; }
tail -2 gpurun_out/r3c_bnb2_tests.log
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3c_bench_bnb2.log 2>&1 || { tail -20 gpurun_out/r3c_bench_bnb2.log; exit 1; }
tail -1 gpurun_out/r3c_bench_bnb2.log | cut -c1-200
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3c_prof_bnb" -o run -- python3 "$R/bench.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3c_prof_bnb.log" 2>&1 || { tail -5 "$R/gpurun_out/r3c_prof_bnb.log"; exit 1; }
cd "$R" && python3 tools/prof_steplist.py gpurun_out/r3c_prof_bnb/run_results.db > gpurun_out/r3c_bnb_steplist.txt && python3 tools/prof_laststep.py gpurun_out/r3c_prof_bnb/run_results.db --top 45 > gpurun_out/r3c_bnb_step.txt && rm -f gpurun_out/r3c_prof_bnb/run_results.db && head -30 gpurun_out/r3c_bnb_step.txt
