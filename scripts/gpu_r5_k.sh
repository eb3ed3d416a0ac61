#!/bin/bash
# r5: ResNet-50 bs1024 eager vs HIP-graph replay, and graph replay under the CLR graph-execution switches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
run() {
  timeout -k 10 300 env "$@" python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5k_b.log 2>&1 || { tail -20 gpurun_out/r5k_b.log; return 1; }
  echo "$*: $(tail -1 gpurun_out/r5k_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d[\"value\"], d[\"ms_per_step\"], d[\"config\"][\"hip_graph\"])")" | tee -a gpurun_out/r5k.log
}
run BENCH_GRAPH=0 && run BENCH_GRAPH=1 && run BENCH_GRAPH=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && run BENCH_GRAPH=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 && run BENCH_GRAPH=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 && run BENCH_GRAPH=0
