#!/bin/bash
# Round-4: batch-1024 step variants: eager (default), HIP graph, high-priority main stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4v_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4v_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step eager 400 python3 bench.py --steps 20 --warmup 5
step graph 400 python3 bench.py --steps 20 --warmup 5 --graph 1
export DL4J_AMD_MAIN_PRIO=1
step prio 400 python3 bench.py --steps 20 --warmup 5
