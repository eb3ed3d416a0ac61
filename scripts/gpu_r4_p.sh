#!/bin/bash
# Round-4: large-batch numerics (repeated-batch score trajectories), then LeNet-MNIST on the GPU: timing at
# warmup 5, kernel trace, host profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4p_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4p_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step dup512 400 python3 tools/batch_dup_check.py --batch 512 --repeat 2 --steps 8
step dup1024 500 python3 tools/batch_dup_check.py --batch 1024 --repeat 2 --steps 6
step lenet 300 python3 tools/bench_lenet.py --device cuda --steps 50 --warmup 5
step lenet_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p_prof -o lenet -- python3 tools/bench_lenet.py --device cuda --steps 50 --warmup 5
step lenet_cprof 300 python3 -m cProfile -s tottime tools/bench_lenet.py --device cuda --steps 50 --warmup 5
head -60 gpurun_out/r4p_lenet_cprof.log
find gpurun_out/r4p_prof -name "*kernel_stats.csv" | head -3
