#!/bin/bash
# r5: BN-backward statistics in the bwd-data epilogue (DL4J_AMD_BN_BWD_EPILOGUE 0/1/2) on the current kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for m in 0 1 2 0; do
  DL4J_AMD_BN_BWD_EPILOGUE=$m timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5o_b.log 2>&1 || { tail -20 gpurun_out/r5o_b.log; exit 1; }
  echo "bnb=$m: $(tail -1 gpurun_out/r5o_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r5o.log
done
