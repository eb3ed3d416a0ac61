#!/bin/bash
# r5: eager vs HIP-graph replay of the ResNet-50 step at bs512 and bs1024 (side stream on in eager mode)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
j() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("hip_graph"))'; }
for b in 512 1024; do
  for g in 0 1; do
    timeout -k 10 240 python3 bench.py --batch $b --graph $g > gpurun_out/r5ak_b${b}_g${g}.log 2>&1 || { tail -5 gpurun_out/r5ak_b${b}_g${g}.log; exit 1; }
    echo "bs$b graph=$g $(j gpurun_out/r5ak_b${b}_g${g}.log)"
  done
done
