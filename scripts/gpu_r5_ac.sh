#!/bin/bash
# r5: multi-rank rehearsal of the torchrun bench path on one GPU (2 ranks, gloo carries the gradient all-reduce) +
# in-process world-1 path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DL4J_AMD_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --batch 128 > gpurun_out/r5ac_tr2.log 2>&1 || { tail -20 gpurun_out/r5ac_tr2.log; exit 1; }
grep '"metric"' gpurun_out/r5ac_tr2.log | cut -c1-400
timeout -k 10 300 python3 bench.py --gpus 1 --inprocess 1 --steps 10 --warmup 3 > gpurun_out/r5ac_inproc1.log 2>&1 || { tail -20 gpurun_out/r5ac_inproc1.log; exit 1; }
grep '"metric"' gpurun_out/r5ac_inproc1.log | cut -c1-300
