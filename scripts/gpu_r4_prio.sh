#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/r4_prio_eager0.log 2>&1 || exit 1; echo "eager prio0 $(tail -1 gpurun_out/r4_prio_eager0.log | cut -c80-140)"
DL4J_AMD_MAIN_PRIO=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/r4_prio_eager1.log 2>&1 || exit 1; echo "eager prio1 $(tail -1 gpurun_out/r4_prio_eager1.log | cut -c80-140)"
done
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4_prio_graph0.log 2>&1 || exit 1; echo "graph prio0 $(tail -1 gpurun_out/r4_prio_graph0.log | cut -c80-140)"
DL4J_AMD_MAIN_PRIO=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4_prio_graph1.log 2>&1 || exit 1; echo "graph prio1 $(tail -1 gpurun_out/r4_prio_graph1.log | cut -c80-140)"
