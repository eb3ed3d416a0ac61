#!/bin/bash
# Full GPU suite, ResNet-50 bench + last-step kernel table, BERT bench, LSTM bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 480 python3 -u -m pytest tests -x -q -m gpu -rs --timeout 120 --timeout-method thread > gpurun_out/r3c_suite_final.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r3c_suite_final.log | head -30; tail -5 gpurun_out/r3c_suite_final.log; exit 1; }
tail -8 gpurun_out/r3c_suite_final.log
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3c_bench_final.log 2>&1 || { tail -20 gpurun_out/r3c_bench_final.log; exit 1; }
tail -1 gpurun_out/r3c_bench_final.log
timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 > gpurun_out/r3c_bench_bert_final.log 2>&1 || { tail -20 gpurun_out/r3c_bench_bert_final.log; exit 1; }
tail -1 gpurun_out/r3c_bench_bert_final.log
timeout -k 10 300 python3 tools/bench_lstm.py > gpurun_out/r3c_bench_lstm_final.log 2>&1 || { tail -20 gpurun_out/r3c_bench_lstm_final.log; exit 1; }
tail -1 gpurun_out/r3c_bench_lstm_final.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3c_prof_zoo_final" -o run -- python3 "$R/bench.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3c_prof_zoo_final.log" 2>&1 || { tail -5 "$R/gpurun_out/r3c_prof_zoo_final.log"; exit 1; }
cd "$R" && python3 tools/prof_steplist.py gpurun_out/r3c_prof_zoo_final/run_results.db > gpurun_out/r3c_zoo_steplist_final.txt && python3 tools/prof_laststep.py gpurun_out/r3c_prof_zoo_final/run_results.db --top 40 > gpurun_out/r3c_zoo_step_final.txt && rm -f gpurun_out/r3c_prof_zoo_final/run_results.db && head -14 gpurun_out/r3c_zoo_step_final.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3c_prof_bert_final" -o run -- python3 "$R/tools/bench_bert.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3c_prof_bert_final.log" 2>&1 || { tail -5 "$R/gpurun_out/r3c_prof_bert_final.log"; exit 1; }
cd "$R" && python3 tools/prof_steplist.py gpurun_out/r3c_prof_bert_final/run_results.db > gpurun_out/r3c_bert_steplist_final.txt && python3 tools/prof_laststep.py gpurun_out/r3c_prof_bert_final/run_results.db --top 30 > gpurun_out/r3c_bert_step_final.txt && rm -f gpurun_out/r3c_prof_bert_final/run_results.db && head -16 gpurun_out/r3c_bert_step_final.txt
