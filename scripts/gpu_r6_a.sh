#!/bin/bash
# r6 baseline: bench twice + kernel-trace profile of the ResNet-50 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py > gpurun_out/r6a_b1.log 2>&1 || { tail -20 gpurun_out/r6a_b1.log; exit 1; }
tail -1 gpurun_out/r6a_b1.log | cut -c1-220
timeout -k 10 300 python3 -u bench.py > gpurun_out/r6a_b2.log 2>&1 || { tail -20 gpurun_out/r6a_b2.log; exit 1; }
tail -1 gpurun_out/r6a_b2.log | cut -c1-220
timeout -k 10 300 python3 tools/gemm_conv1x1_bench.py --cfgs 5,8,9 > gpurun_out/r6a_1x1.log 2>&1 || { tail -20 gpurun_out/r6a_1x1.log; exit 1; }
cat gpurun_out/r6a_1x1.log
bash scripts/prof_resnet.sh r6a_prof && python3 tools/prof_steplist.py gpurun_out/r6a_prof/*/run_results.db > gpurun_out/r6a_steplist.txt 2>&1; tail -2 gpurun_out/r6a_steplist.txt
