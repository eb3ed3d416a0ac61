#!/bin/bash
# r6zd: in-kernel slab reduction tree limited to small split counts (DL4J_AMD_WRW_TREE_MAX) vs the reduce launch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "0 0" "8 16" "8 64" "4 16" "0 0" "8 16" "8 64"; do
  set -- $cfg
  DL4J_AMD_WRW_TREE=$1 DL4J_AMD_WRW_TREE_MAX=$2 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6zd_bench.json 2> gpurun_out/r6zd_bench.err || { tail -5 gpurun_out/r6zd_bench.err; exit 1; }
  echo "fan $1 max $2: $(tail -1 gpurun_out/r6zd_bench.json | cut -c80-140)"
done
