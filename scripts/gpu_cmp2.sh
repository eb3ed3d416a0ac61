#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python -u tools/bench_torch_comparators.py --model resnet50 --nchw 1 --steps 5 --warmup 2 > gpurun_out/cmp_torch_resnet_nchw.log 2> gpurun_out/cmp_torch_resnet_nchw.err; tail -1 gpurun_out/cmp_torch_resnet_nchw.log
