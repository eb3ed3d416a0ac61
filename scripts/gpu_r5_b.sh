#!/bin/bash
# r5: fixed per-tile cost vs per-K-tile cost of the in-tree GEMM configs (K scan), bf16 and fp32 outputs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/gemm_probe.py --M 4096 --N 2304 --ks 64,128,256,512,768,1536,3072 --cfgs 4,2,3,0 --outs bf16,fp32 > gpurun_out/r5b_probe.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/gemm_probe.py --M 4096 --N 4096 --ks 64,128,256,512,1024,2048,4096 --cfgs 4,2 --outs bf16 >> gpurun_out/r5b_probe.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5b_probe.log
