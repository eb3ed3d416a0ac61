#!/bin/bash
# Round-4: attention forward with two key blocks staged per round (D = 64). Attention / transformer / SameDiff tests,
# BERT CG + SameDiff benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4m_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4m_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step t_attn 300 $PT tests/test_gpu_transformer.py tests/test_gpu_self_attention.py tests/test_gpu_samediff.py
step b_bert 300 python3 tools/bench_bert.py --steps 10 --warmup 3
step b_bert_sd 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3
step b_bert16 300 python3 tools/bench_bert.py --steps 10 --warmup 3 --dtype fp16
step b_bert_sd16 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3 --dtype fp16
