#!/bin/bash
# r5: 1x1-conv GEMM shapes (canonical stage 2 at batch 512 / zoo stage 2 at batch 1024), per config
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for s in "--M 1605632 --N 256 --ks 64" "--M 1605632 --N 64 --ks 256" "--M 802816 --N 256 --ks 64" "--M 802816 --N 128 --ks 512" "--M 200704 --N 512 --ks 128"; do
  timeout -k 10 200 python3 -u tools/gemm_probe.py $s --cfgs 0,1,2,3,4,5,6 --outs bf16 >> gpurun_out/r5n_probe.log 2>&1 || { tail -5 gpurun_out/r5n_probe.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r5n_probe.log
