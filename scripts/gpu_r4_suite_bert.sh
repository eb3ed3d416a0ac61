#!/bin/bash
# Full GPU suite on the current tree, then BERT: GEMM table vs torch, CG bench graph / eager, SameDiff bench + kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu -rs --timeout 150 --timeout-method thread > gpurun_out/r4_suite.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r4_suite.log | head -30; tail -30 gpurun_out/r4_suite.log; exit 1; }
tail -3 gpurun_out/r4_suite.log
timeout -k 10 300 python3 tools/gemm_bench.py > gpurun_out/r4_gemm_bench.log 2>&1 || { tail -20 gpurun_out/r4_gemm_bench.log; exit 1; }
cat gpurun_out/r4_gemm_bench.log | grep -v amdgpu.ids
timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 > gpurun_out/r4_bert_graph.log 2>&1 || { tail -20 gpurun_out/r4_bert_graph.log; exit 1; }
echo "bert graph: $(tail -1 gpurun_out/r4_bert_graph.log | cut -c1-160)"
timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 --graph 0 > gpurun_out/r4_bert_eager.log 2>&1 || { tail -20 gpurun_out/r4_bert_eager.log; exit 1; }
echo "bert eager: $(tail -1 gpurun_out/r4_bert_eager.log | cut -c1-160)"
timeout -k 10 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3 > gpurun_out/r4_bert_sd.log 2>&1 || { tail -20 gpurun_out/r4_bert_sd.log; exit 1; }
echo "bert samediff: $(tail -1 gpurun_out/r4_bert_sd.log | cut -c1-160)"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4_sd_prof" -o run -- python3 "$R/tools/bench_bert_samediff.py" --steps 4 --warmup 3 > "$R/gpurun_out/r4_sd_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r4_sd_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r4_sd_prof/run_results.db --top 40 > gpurun_out/r4_sd_step.txt && rm -rf gpurun_out/r4_sd_prof && head -30 gpurun_out/r4_sd_step.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4_eager_prof" -o run -- python3 "$R/bench.py" --steps 4 --warmup 3 > "$R/gpurun_out/r4_eager_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r4_eager_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r4_eager_prof/run_results.db --top 45 > gpurun_out/r4_eager_step.txt && python3 tools/prof_steplist.py gpurun_out/r4_eager_prof/run_results.db > gpurun_out/r4_eager_steplist.txt && rm -rf gpurun_out/r4_eager_prof && head -30 gpurun_out/r4_eager_step.txt
