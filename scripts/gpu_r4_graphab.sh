#!/bin/bash
# Eager vs HIP-graph replay of the ResNet-50 step, with and without the weight-gradient overlap stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { # tag env... -- args
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 $BARGS > gpurun_out/r4_gab_$tag.log 2>&1 || { tail -5 gpurun_out/r4_gab_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/r4_gab_$tag.log | cut -c80-140)"
}
BARGS="--graph 0" run eager_ws1 DL4J_AMD_WRW_STREAM=1
BARGS="--graph 0" run eager_ws0 DL4J_AMD_WRW_STREAM=0
BARGS="--graph 1" run graph_ws1 DL4J_AMD_WRW_STREAM=1
BARGS="--graph 1" run graph_ws0 DL4J_AMD_WRW_STREAM=0
BARGS="--graph 0" run eager_ws1b DL4J_AMD_WRW_STREAM=1
BARGS="--graph 0 --variant canonical" run canon_eager DL4J_AMD_WRW_STREAM=1
BARGS="--graph 1 --variant canonical" run canon_graph DL4J_AMD_WRW_STREAM=1
