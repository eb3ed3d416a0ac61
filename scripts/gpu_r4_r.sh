#!/bin/bash
# Round-4: repeated-batch gradient check of the ResNet-50 bench path at per-GPU batch 64 -> 2048.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4r_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4r_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step dup64 300 python3 tools/batch_dup_check.py --batch 64 --repeat 2 --steps 1
step dup512 300 python3 tools/batch_dup_check.py --batch 512 --repeat 2 --steps 1
step dup1024 400 python3 tools/batch_dup_check.py --batch 1024 --repeat 2 --steps 1
