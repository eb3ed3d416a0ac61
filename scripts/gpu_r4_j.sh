#!/bin/bash
# Round-4: SameDiff residual-gradient accumulation inside the linear's dX GEMM. Tests, SameDiff / CG BERT, ResNet x2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4j_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4j_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step t_sd 300 $PT tests/test_gpu_samediff.py tests/test_gpu_transformer.py
step b_bert_sd 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3
step b_bert_sd_noacc 300 env DL4J_AMD_SD_ACC=0 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3
step b_bert 300 python3 tools/bench_bert.py --steps 10 --warmup 3
step b_bert_sd16 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3 --dtype fp16
step b_resnet1 400 python3 bench.py --steps 30 --warmup 5
step b_resnet2 400 python3 bench.py --steps 30 --warmup 5
