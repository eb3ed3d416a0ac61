#!/bin/bash
# r5: benches with the recorded gfx950 kernel-choice database vs per-process autotuning (DL4J_AMD_TUNE_DB=off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
j() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for db in on off on; do
  if [ $db = off ]; then export DL4J_AMD_TUNE_DB=off; else unset DL4J_AMD_TUNE_DB; fi
  timeout -k 10 200 python3 bench.py > gpurun_out/r5ae_zoo_$db.log 2>&1 || { tail -5 gpurun_out/r5ae_zoo_$db.log; exit 1; }
  echo "zoo db=$db $(j gpurun_out/r5ae_zoo_$db.log)"
  timeout -k 10 300 python3 tools/bench_bert.py > gpurun_out/r5ae_bert_$db.log 2>&1 || { tail -5 gpurun_out/r5ae_bert_$db.log; exit 1; }
  echo "bert db=$db $(j gpurun_out/r5ae_bert_$db.log)"
  timeout -k 10 200 python3 bench.py --variant canonical --batch 512 --steps 15 --warmup 4 > gpurun_out/r5ae_canon_$db.log 2>&1 || { tail -5 gpurun_out/r5ae_canon_$db.log; exit 1; }
  echo "canon db=$db $(j gpurun_out/r5ae_canon_$db.log)"
  timeout -k 10 300 python3 bench.py --gpus 1 --inprocess 1 > gpurun_out/r5ae_inproc_$db.log 2>&1 || { tail -5 gpurun_out/r5ae_inproc_$db.log; exit 1; }
  echo "inprocess world-1 db=$db $(j gpurun_out/r5ae_inproc_$db.log)"
done
