#!/bin/bash
# BN relu bitmask + fused fold/finalize; LSTM window launch trimming. Numerics, then benches + last-step profiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_conv.py tests/test_gpu_bnpool.py tests/test_gpu_lstm.py tests/test_gpu_gemm.py tests/test_gpu_transformer.py -x -v --timeout 300 --timeout-method thread -k "batchnorm or bn or resnet or lstm or gemm or softmax or lenet or layernorm or bert" > gpurun_out/r3_tests_bnlstm.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3_tests_bnlstm.log | head -30; tail -5 gpurun_out/r3_tests_bnlstm.log; exit 1; }
tail -2 gpurun_out/r3_tests_bnlstm.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_bn.log 2>&1 || { tail -20 gpurun_out/r3_bench_bn.log; exit 1; }
tail -1 gpurun_out/r3_bench_bn.log
DL4J_AMD_BN_FOLD=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_bn_nofold.log 2>&1 || { tail -20 gpurun_out/r3_bench_bn_nofold.log; exit 1; }
tail -1 gpurun_out/r3_bench_bn_nofold.log
timeout -k 10 300 python3 tools/bench_lstm.py --steps 5 --warmup 2 > gpurun_out/r3_bench_lstm2.log 2>&1 || { tail -20 gpurun_out/r3_bench_lstm2.log; exit 1; }
tail -1 gpurun_out/r3_bench_lstm2.log
DL4J_AMD_LSTM_COOP_LAUNCH=coop timeout -k 10 300 python3 tools/bench_lstm.py --steps 5 --warmup 2 > gpurun_out/r3_bench_lstm2_cooplaunch.log 2>&1 || { tail -20 gpurun_out/r3_bench_lstm2_cooplaunch.log; exit 1; }
tail -1 gpurun_out/r3_bench_lstm2_cooplaunch.log
timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 > gpurun_out/r3_bench_bert2.log 2>&1 || { tail -20 gpurun_out/r3_bench_bert2.log; exit 1; }
tail -1 gpurun_out/r3_bench_bert2.log
DL4J_AMD_LN_BWD=wave timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 > gpurun_out/r3_bench_bert2_lnwave.log 2>&1 || { tail -20 gpurun_out/r3_bench_bert2_lnwave.log; exit 1; }
tail -1 gpurun_out/r3_bench_bert2_lnwave.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3_prof_bn" -o run -- python3 "$R/bench.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3_prof_bn.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_prof_bn.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r3_prof_bn/run_results.db --top 45 > gpurun_out/r3_prof_bn_step.txt && rm -f gpurun_out/r3_prof_bn/run_results.db && head -30 gpurun_out/r3_prof_bn_step.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3_prof_lstm2" -o run -- python3 "$R/tools/bench_lstm.py" --steps 3 --warmup 2 > "$R/gpurun_out/r3_prof_lstm2.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_prof_lstm2.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r3_prof_lstm2/run_results.db --top 40 > gpurun_out/r3_prof_lstm2_step.txt && python3 tools/prof_steplist.py gpurun_out/r3_prof_lstm2/run_results.db > gpurun_out/r3_prof_lstm2_list.txt && rm -f gpurun_out/r3_prof_lstm2/run_results.db && head -25 gpurun_out/r3_prof_lstm2_step.txt
