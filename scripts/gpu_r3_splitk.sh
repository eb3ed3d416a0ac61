#!/bin/bash
# channel_sum_reduce with eight loads per trip: tests, BERT bench, BERT last-step kernel table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_transformer.py tests/test_gpu_lstm.py -x -q -rs --timeout 120 --timeout-method thread > gpurun_out/r3c_splitk_tests.log 2>&1 || { tail -40 gpurun_out/r3c_splitk_tests.log; exit 1; }
tail -1 gpurun_out/r3c_splitk_tests.log
timeout -k 10 240 python3 tools/bench_bert.py --steps 10 --warmup 3 > gpurun_out/r3c_bench_bert_splitk.log 2>&1 || { tail -20 gpurun_out/r3c_bench_bert_splitk.log; exit 1; }
tail -1 gpurun_out/r3c_bench_bert_splitk.log | cut -c1-160
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3c_prof_bert_splitk" -o run -- python3 "$R/tools/bench_bert.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3c_prof_bert_splitk.log" 2>&1 || { tail -5 "$R/gpurun_out/r3c_prof_bert_splitk.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r3c_prof_bert_splitk/run_results.db --top 30 > gpurun_out/r3c_bert_step_splitk.txt && rm -f gpurun_out/r3c_prof_bert_splitk/run_results.db && grep -E "one step|splitk" gpurun_out/r3c_bert_step_splitk.txt
