#!/bin/bash
# Round-4 combined validation: stacked LSTM, SameDiff gradient sinks, GEMM library candidate, tiled weight relayout;
# then the LSTM / SameDiff / BERT / GEMM / ResNet benches. A failing test is recorded and the run goes on; a crash,
# abort or time limit ends it (no further GPU step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/r4c_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "gpurun_out/r4c_$name.log" | tail -1 | cut -c1-220)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step t_stack 300 $PT tests/test_gpu_lstm_stack.py
step t_lstm 300 $PT tests/test_gpu_lstm.py
step t_sd 300 $PT tests/test_gpu_samediff.py
step t_gemm 300 $PT tests/test_gpu_gemm.py
step t_conv 400 $PT tests/test_gpu_conv.py tests/test_gpu_conv_v3.py
step b_lstm 300 python3 tools/bench_lstm.py --steps 5 --warmup 2
step b_lstm_nostack 300 env DL4J_AMD_LSTM_STACK=0 python3 tools/bench_lstm.py --steps 5 --warmup 2
step b_sdlstm 300 python3 tools/bench_samediff_lstm.py
step b_gemm 300 python3 tools/gemm_bench.py --rounds 3
step b_bert 300 python3 tools/bench_bert.py --steps 10 --warmup 3
step b_bert_sd 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3
step b_resnet 400 python3 bench.py --steps 30 --warmup 5
grep -v amdgpu.ids gpurun_out/r4c_b_gemm.log
