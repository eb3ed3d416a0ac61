#!/bin/bash
# r5: A/B on one box — lean epilogue on/off and library GEMM candidate on/off (ResNet-50 bs1024, BERT)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "1 1" "0 1" "1 0" "1 1" "0 0"; do
  set -- $cfg
  DL4J_AMD_GEMM_LEAN=$1 DL4J_AMD_GEMM_LIB=$2 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5h_b.log 2>&1 || { tail -20 gpurun_out/r5h_b.log; exit 1; }
  echo "resnet lean=$1 lib=$2: $(tail -1 gpurun_out/r5h_b.log | cut -c1-140)" | tee -a gpurun_out/r5h.log
done
for lib in 1 0; do
  DL4J_AMD_GEMM_LIB=$lib timeout -k 10 300 python3 tools/bench_bert.py --steps 10 --warmup 3 > gpurun_out/r5h_bert.log 2>&1 || { tail -20 gpurun_out/r5h_bert.log; exit 1; }
  echo "bert lib=$lib: $(tail -1 gpurun_out/r5h_bert.log | cut -c1-120)" | tee -a gpurun_out/r5h.log
done
