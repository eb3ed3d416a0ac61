#!/bin/bash
# r5: secondary benchmarks on the in-tree-only defaults: LSTM (CG + SameDiff), BERT fp16, LeNet eager, canonical
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
j() { tail -1 "$1" | cut -c1-190; }
timeout -k 10 300 python3 tools/bench_lstm.py > gpurun_out/r5p_lstm.log 2>&1 || { tail -20 gpurun_out/r5p_lstm.log; exit 1; }
echo "lstm: $(j gpurun_out/r5p_lstm.log)" | tee gpurun_out/r5p.log
timeout -k 10 300 python3 tools/bench_samediff_lstm.py > gpurun_out/r5p_sdlstm.log 2>&1 || { tail -20 gpurun_out/r5p_sdlstm.log; exit 1; }
echo "samediff lstm: $(j gpurun_out/r5p_sdlstm.log)" | tee -a gpurun_out/r5p.log
timeout -k 10 300 python3 tools/bench_bert.py --dtype fp16 --steps 10 --warmup 3 > gpurun_out/r5p_bert16.log 2>&1 || { tail -20 gpurun_out/r5p_bert16.log; exit 1; }
echo "bert fp16: $(j gpurun_out/r5p_bert16.log)" | tee -a gpurun_out/r5p.log
timeout -k 10 300 python3 tools/bench_lenet.py --device cuda --graph 0 > gpurun_out/r5p_lenet.log 2>&1 || { tail -20 gpurun_out/r5p_lenet.log; exit 1; }
echo "lenet eager: $(j gpurun_out/r5p_lenet.log)" | tee -a gpurun_out/r5p.log
DL4J_AMD_GEMM_LIB=1 timeout -k 10 300 python3 tools/bench_lenet.py --device cuda > gpurun_out/r5p_lenet_lib.log 2>&1 || { tail -20 gpurun_out/r5p_lenet_lib.log; exit 1; }
echo "lenet graph lib-opt-in: $(j gpurun_out/r5p_lenet_lib.log)" | tee -a gpurun_out/r5p.log
