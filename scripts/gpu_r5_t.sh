#!/bin/bash
# r5: weight-gradient side stream on/off, zoo bs1024 and canonical bs512
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
j() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for w in 0 1; do
  DL4J_AMD_WRW_STREAM=$w timeout -k 10 200 python3 bench.py --steps 15 --warmup 4 > gpurun_out/r5t_zoo_$w.log 2>&1 || { tail -5 gpurun_out/r5t_zoo_$w.log; exit 1; }
  echo "zoo wrw_stream=$w $(j gpurun_out/r5t_zoo_$w.log)"
  DL4J_AMD_WRW_STREAM=$w timeout -k 10 200 python3 bench.py --variant canonical --batch 512 --steps 15 --warmup 4 > gpurun_out/r5t_canon_$w.log 2>&1 || { tail -5 gpurun_out/r5t_canon_$w.log; exit 1; }
  echo "canon wrw_stream=$w $(j gpurun_out/r5t_canon_$w.log)"
done
