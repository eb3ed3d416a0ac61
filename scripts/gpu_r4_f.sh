#!/bin/bash
# Round-4: library GEMM candidate for epilogue call sites (bias shadow kept through layers' matmul, activation /
# dgelu epilogues as library product + in-tree elementwise kernel), graph-replay input cast, TBPTT state foreach copy.
# Tests first, then the epilogue GEMM table and the BERT / SameDiff / LSTM / ResNet benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4f_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4f_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step t_gemm 300 $PT tests/test_gpu_gemm.py
step t_tr 300 $PT tests/test_gpu_transformer.py tests/test_gpu_samediff.py tests/test_gpu_lstm_graph.py tests/test_gpu_lstm_stack.py
step b_epi 300 python3 tools/gemm_bench.py --epilogues-only --rounds 3
grep -v amdgpu.ids gpurun_out/r4f_b_epi.log
step b_bert 300 python3 tools/bench_bert.py --steps 10 --warmup 3
step b_bert_sd 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3
step b_lstm 300 python3 tools/bench_lstm.py --steps 5 --warmup 2
step b_sdlstm 300 python3 tools/bench_samediff_lstm.py
step b_resnet 400 python3 bench.py --steps 30 --warmup 5
