#!/bin/bash
# Round-3 baseline: bench, kernel-trace profile and one PMC pass (MFMA / LDS counters) of the ResNet-50 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_base.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r3_bench_base.log; exit 1; }
tail -1 gpurun_out/r3_bench_base.log
bash scripts/prof_resnet.sh r3_prof_base || exit 1
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d "$R/gpurun_out/r3_pmc_base" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --graph 0 > "$R/gpurun_out/r3_pmc_base.log" 2>&1
rc=$?; cd "$R"; [ $rc -eq 0 ] && echo PMC_OK || { echo "PMC_FAIL rc=$rc"; tail -5 gpurun_out/r3_pmc_base.log; exit 1; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv_safety.py tests/test_gpu_dist.py tests/test_gpu_conv.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_tests_safety.log 2>&1; rc=$?
tail -5 gpurun_out/r3_tests_safety.log; exit $rc
