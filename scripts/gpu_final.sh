#!/bin/bash
# Full GPU suite + smoke, then a 2-rank DP rehearsal (gloo, both ranks on the one GPU; exercises the bucketed
# all-reduce + weight-gradient overlap stream joins), then the default bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
bash scripts/gpu_full.sh || exit 1
DL4J_AMD_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --batch 64 --steps 5 --warmup 2 > gpurun_out/dp2_gloo.log 2>&1 || { tail -30 gpurun_out/dp2_gloo.log; exit 1; }
grep '"metric"' gpurun_out/dp2_gloo.log | cut -c1-250
timeout -k 10 300 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log
