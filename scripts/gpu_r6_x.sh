#!/bin/bash
# r6x: re-time the zoo ResNet-50 bs1024 kernel choices with the round-6 kernels (1x1 GEMM-vs-implicit, conv variants
# incl. stream / halo, GEMM configs, weight-gradient splits) and compare against the shipped database on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
rm -f gpurun_out/r6x_tune_zoo.json
DL4J_AMD_TUNE_DB_SKIP=conv_1x1,conv_v3,gemm,conv_wrw DL4J_AMD_TUNE_RECORD=$R/gpurun_out/r6x_tune_zoo.json DL4J_AMD_TUNE_REPS=6 timeout -k 10 500 python3 -u bench.py > gpurun_out/r6x_bench_retune.log 2>&1 || { tail -20 gpurun_out/r6x_bench_retune.log; exit 1; }
tail -1 gpurun_out/r6x_bench_retune.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py > gpurun_out/r6x_bench_db.log 2>&1 || { tail -20 gpurun_out/r6x_bench_db.log; exit 1; }
tail -1 gpurun_out/r6x_bench_db.log | cut -c1-200
DL4J_AMD_TUNE_DB=$R/gpurun_out/r6x_tune_zoo.json timeout -k 10 300 python3 -u bench.py > gpurun_out/r6x_bench_rec.log 2>&1 || { tail -20 gpurun_out/r6x_bench_rec.log; exit 1; }
tail -1 gpurun_out/r6x_bench_rec.log | cut -c1-200
