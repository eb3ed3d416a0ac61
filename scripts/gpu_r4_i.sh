#!/bin/bash
# Round-4: stem weight gradient with a swizzled transposed dy tile (no 8-way LDS write conflicts); bnpool backward
# reverted. Stem tests, stem kernel timings, ResNet bench twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4i_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4i_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step t_stem 300 $PT tests/test_gpu_bnpool.py
step stem 300 python3 tools/stem_bench.py
grep -v amdgpu.ids gpurun_out/r4i_stem.log
step b_resnet1 400 python3 bench.py --steps 30 --warmup 5
step b_resnet2 400 python3 bench.py --steps 30 --warmup 5
step b_bert_sd 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3
step b_bert 300 python3 tools/bench_bert.py --steps 10 --warmup 3
