#!/bin/bash
# Round-4: kernel trace of the ResNet-50 step at the default per-GPU batch 1024.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4u_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4u_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r4u_prof -o resnet1024 -- python3 bench.py --steps 3 --warmup 4
