#!/bin/bash
# Round-4 closing validation of the final tree:
# full GPU suite, smoke, default bench, BERT / SameDiff / LSTM benches, LeNet-MNIST on the GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4x_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4x_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
step suite 900 python3 -u -m pytest tests -q -m gpu -rs --maxfail 5 --timeout 150 --timeout-method thread
grep -E "^FAILED|^ERROR" gpurun_out/r4x_suite.log | head -20
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python3 bench.py
step b_sd16 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3 --dtype fp16
step b_sd 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3
step b_bert16 300 python3 tools/bench_bert.py --steps 10 --warmup 3 --dtype fp16
step b_lstm 300 python3 tools/bench_lstm.py --steps 5 --warmup 2
step b_lenet 300 python3 tools/bench_lenet.py --device cuda --steps 50 --warmup 5
step b_sdlstm 300 python3 tools/bench_samediff_lstm.py
