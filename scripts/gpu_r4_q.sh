#!/bin/bash
# Round-4: ResNet-50 per-GPU batch sweep above 1024 (peak memory in the JSON config).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4q_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4q_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step b1024 500 python3 bench.py --steps 20 --warmup 5 --batch 1024
step b1536 600 python3 bench.py --steps 15 --warmup 5 --batch 1536
step b2048 700 python3 bench.py --steps 10 --warmup 5 --batch 2048
