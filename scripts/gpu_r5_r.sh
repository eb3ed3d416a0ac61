#!/bin/bash
# r5: CU-masked weight-gradient side stream sweep (canonical bs512, zoo bs1024)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 python3 -c "
import torch
from deeplearning4j_amd import runtime as rt
s = rt.Stream(0, cus=192); print('cu_count masked', s.cu_count())
t = rt.Stream(0); print('cu_count plain', t.cu_count())
" > gpurun_out/r5r_mask.txt 2>&1 || { cat gpurun_out/r5r_mask.txt; exit 1; }
cat gpurun_out/r5r_mask.txt
for cus in 0 224 192 160; do
  DL4J_AMD_WRW_CUS=$cus timeout -k 10 200 python3 bench.py --variant canonical --batch 512 --steps 15 --warmup 4 > gpurun_out/r5r_canon_$cus.log 2>&1 || { tail -5 gpurun_out/r5r_canon_$cus.log; exit 1; }
  echo "canon cus=$cus $(tail -1 gpurun_out/r5r_canon_$cus.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
for cus in 0 224 192 160; do
  DL4J_AMD_WRW_CUS=$cus timeout -k 10 200 python3 bench.py --steps 15 --warmup 4 > gpurun_out/r5r_zoo_$cus.log 2>&1 || { tail -5 gpurun_out/r5r_zoo_$cus.log; exit 1; }
  echo "zoo cus=$cus $(tail -1 gpurun_out/r5r_zoo_$cus.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
