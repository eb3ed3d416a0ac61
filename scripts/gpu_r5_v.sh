#!/bin/bash
# r5: BERT GEMM autotune candidate times per call site (us)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DL4J_AMD_GEMM_TUNE_LOG=1 timeout -k 10 300 python3 tools/bench_bert.py --steps 3 --warmup 2 > gpurun_out/r5v_bert_tune.log 2>&1 || { tail -5 gpurun_out/r5v_bert_tune.log; exit 1; }
grep gemm-tune gpurun_out/r5v_bert_tune.log | cut -c1-250
tail -1 gpurun_out/r5v_bert_tune.log | cut -c1-200
