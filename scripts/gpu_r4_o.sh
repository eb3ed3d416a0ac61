#!/bin/bash
# Round-4: ResNet-50 per-GPU batch sweep (512 / 768 / 1024) with the default eager bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4o_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4o_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step b512 400 python3 bench.py --steps 30 --warmup 5 --batch 512
step b768 400 python3 bench.py --steps 20 --warmup 5 --batch 768
step b1024 500 python3 bench.py --steps 15 --warmup 5 --batch 1024
step b640 400 python3 bench.py --steps 25 --warmup 5 --batch 640
