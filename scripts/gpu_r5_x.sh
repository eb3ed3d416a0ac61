#!/bin/bash
# r5: HBM write ceiling probe + 1x1-conv GEMMs with non-temporal output stores
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/hbm_probe.py > gpurun_out/r5x_hbm.txt 2>&1 || { cat gpurun_out/r5x_hbm.txt; exit 1; }
cat gpurun_out/r5x_hbm.txt
timeout -k 10 120 python3 tools/hbm_probe.py --mb 64 >> gpurun_out/r5x_hbm.txt 2>&1 || exit 1
tail -4 gpurun_out/r5x_hbm.txt
for nt in 0 1; do
  DL4J_AMD_GEMM_STORE_NT=$nt timeout -k 10 300 python3 tools/gemm_conv1x1_bench.py --cfgs 5,8,9 > gpurun_out/r5x_conv1x1_nt$nt.txt 2>&1 || { tail -5 gpurun_out/r5x_conv1x1_nt$nt.txt; exit 1; }
  echo "store_nt=$nt"; cat gpurun_out/r5x_conv1x1_nt$nt.txt
done
j() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for nt in 0 1; do
  DL4J_AMD_GEMM_STORE_NT=$nt timeout -k 10 200 python3 bench.py --steps 15 --warmup 4 > gpurun_out/r5x_zoo_nt$nt.log 2>&1 || { tail -5 gpurun_out/r5x_zoo_nt$nt.log; exit 1; }
  echo "zoo store_nt=$nt $(j gpurun_out/r5x_zoo_nt$nt.log)"
done
