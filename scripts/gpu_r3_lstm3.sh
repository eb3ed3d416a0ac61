#!/bin/bash
# LSTM device-side coop tags / fp32 bias / no grad fill; BERT dgelu epilogue + LN dsum. Tests, benches, profiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_gemm.py tests/test_gpu_transformer.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3_tests_lstm3.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3_tests_lstm3.log | head -30; tail -5 gpurun_out/r3_tests_lstm3.log; exit 1; }
tail -2 gpurun_out/r3_tests_lstm3.log
timeout -k 10 300 python3 tools/bench_lstm.py --steps 5 --warmup 2 > gpurun_out/r3_bench_lstm3.log 2>&1 || { tail -20 gpurun_out/r3_bench_lstm3.log; exit 1; }
tail -1 gpurun_out/r3_bench_lstm3.log
timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 > gpurun_out/r3_bench_bert3.log 2>&1 || { tail -20 gpurun_out/r3_bench_bert3.log; exit 1; }
tail -1 gpurun_out/r3_bench_bert3.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3_prof_lstm3" -o run -- python3 "$R/tools/bench_lstm.py" --steps 3 --warmup 2 > "$R/gpurun_out/r3_prof_lstm3.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_prof_lstm3.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r3_prof_lstm3/run_results.db --top 40 > gpurun_out/r3_prof_lstm3_step.txt && python3 tools/prof_steplist.py gpurun_out/r3_prof_lstm3/run_results.db > gpurun_out/r3_prof_lstm3_list.txt && rm -f gpurun_out/r3_prof_lstm3/run_results.db && head -20 gpurun_out/r3_prof_lstm3_step.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3_prof_bert3" -o run -- python3 "$R/tools/bench_bert.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3_prof_bert3.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_prof_bert3.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r3_prof_bert3/run_results.db --top 40 > gpurun_out/r3_prof_bert3_step.txt && rm -f gpurun_out/r3_prof_bert3/run_results.db && head -30 gpurun_out/r3_prof_bert3_step.txt
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_conv.py -x -q --timeout 300 --timeout-method thread -k "batchnorm or bn_stats or resnet" > gpurun_out/r3_tests_bn3.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3_tests_bn3.log | head -30; tail -5 gpurun_out/r3_tests_bn3.log; exit 1; }
tail -1 gpurun_out/r3_tests_bn3.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_bn3.log 2>&1 || { tail -20 gpurun_out/r3_bench_bn3.log; exit 1; }
tail -1 gpurun_out/r3_bench_bn3.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3_prof_bn3" -o run -- python3 "$R/bench.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3_prof_bn3.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_prof_bn3.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r3_prof_bn3/run_results.db --top 45 > gpurun_out/r3_prof_bn3_step.txt && rm -f gpurun_out/r3_prof_bn3/run_results.db && grep -E "bn_|one step" gpurun_out/r3_prof_bn3_step.txt
