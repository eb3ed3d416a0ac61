#!/bin/bash
# GEMM library candidate + SameDiff gradient sinks: focused GPU tests, GEMM table with the dispatch pick, BERT CG
# (graph / eager) and SameDiff benches, SameDiff one-step kernel table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_samediff.py tests/test_gpu_gemm.py tests/test_gpu_transformer.py tests/test_gpu_kernels.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r4_lib_tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r4_lib_tests.log | head -30; tail -30 gpurun_out/r4_lib_tests.log; exit 1; }
tail -2 gpurun_out/r4_lib_tests.log
timeout -k 10 300 python3 tools/gemm_bench.py --rounds 3 > gpurun_out/r4_lib_gemm.log 2>&1 || { tail -20 gpurun_out/r4_lib_gemm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_lib_gemm.log
timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 > gpurun_out/r4_lib_bert_graph.log 2>&1 || { tail -20 gpurun_out/r4_lib_bert_graph.log; exit 1; }
echo "bert graph: $(tail -1 gpurun_out/r4_lib_bert_graph.log | cut -c1-170)"
timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 --graph 0 > gpurun_out/r4_lib_bert_eager.log 2>&1 || { tail -20 gpurun_out/r4_lib_bert_eager.log; exit 1; }
echo "bert eager: $(tail -1 gpurun_out/r4_lib_bert_eager.log | cut -c1-170)"
timeout -k 10 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3 > gpurun_out/r4_lib_bert_sd.log 2>&1 || { tail -20 gpurun_out/r4_lib_bert_sd.log; exit 1; }
echo "bert samediff: $(tail -1 gpurun_out/r4_lib_bert_sd.log | cut -c1-170)"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4_lib_sd_prof" -o run -- python3 "$R/tools/bench_bert_samediff.py" --steps 4 --warmup 3 > "$R/gpurun_out/r4_lib_sd_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r4_lib_sd_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r4_lib_sd_prof/run_results.db --top 40 > gpurun_out/r4_lib_sd_step.txt && rm -rf gpurun_out/r4_lib_sd_prof && head -30 gpurun_out/r4_lib_sd_step.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4_lib_cg_prof" -o run -- python3 "$R/tools/bench_bert.py" --steps 4 --warmup 3 > "$R/gpurun_out/r4_lib_cg_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r4_lib_cg_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r4_lib_cg_prof/run_results.db --top 40 > gpurun_out/r4_lib_cg_step.txt && rm -rf gpurun_out/r4_lib_cg_prof && head -30 gpurun_out/r4_lib_cg_step.txt
