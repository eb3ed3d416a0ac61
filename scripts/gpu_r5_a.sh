#!/bin/bash
# r5 first look: per-config GEMM times on the BERT / square shapes, in-tree vs torch (hipBLASLt)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/gemm_probe.py --M 4096 --N 2304 --ks 768 --cfgs 0,1,2,3,4,5,6,7 --outs bf16 > gpurun_out/r5a_probe.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/gemm_probe.py --M 4096 --N 768 --ks 768,3072 --cfgs 0,1,2,3,4,5,6,7 --outs bf16 >> gpurun_out/r5a_probe.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/gemm_probe.py --M 4096 --N 3072 --ks 768 --cfgs 0,1,2,3,4,5,6,7 --outs bf16 >> gpurun_out/r5a_probe.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/gemm_probe.py --M 4096 --N 4096 --ks 4096 --cfgs 0,1,4 --outs bf16 >> gpurun_out/r5a_probe.log 2>&1 || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5a_prof" -o run -- python3 "$R/tools/gemm_probe.py" --M 4096 --N 2304 --ks 768 --cfgs 4,1 --outs bf16 > "$R/gpurun_out/r5a_prof.log" 2>&1 || exit 1
cd "$R"; ls gpurun_out/r5a_prof
grep -v amdgpu.ids gpurun_out/r5a_probe.log
