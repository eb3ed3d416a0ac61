#!/bin/bash
# r5: epilogue sub-phase stamps of the 8-phase GEMM
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in "4096 2304 64" "4096 2304 768" "4096 768 3072"; do
  timeout -k 5 60 ./tools/native/gemm_stamps $s 4 >> gpurun_out/r5e_stamps.log 2>&1 || exit 1
done
cat gpurun_out/r5e_stamps.log
