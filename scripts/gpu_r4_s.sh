#!/bin/bash
# Round-4: first-pass (autotuning) vs second-pass gradients; fp32 library GEMM candidate tests; LeNet on the GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4s_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4s_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step dup64 300 python3 tools/batch_dup_check.py --batch 64 --repeat 2 --steps 1
step t_gemm 300 $PT tests/test_gpu_gemm.py
step lenet 300 python3 tools/bench_lenet.py --device cuda --steps 50 --warmup 5
