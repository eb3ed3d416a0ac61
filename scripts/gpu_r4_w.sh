#!/bin/bash
# Round-4: LeNet-MNIST on the GPU, eager vs HIP-graph replay (launch-bound step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4w_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4w_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step eager 300 python3 tools/bench_lenet.py --device cuda --steps 100 --warmup 5
step graph 300 python3 tools/bench_lenet.py --device cuda --steps 100 --warmup 5 --graph 1
step t_graph 300 $PT tests/test_gpu_graph_workspace.py
