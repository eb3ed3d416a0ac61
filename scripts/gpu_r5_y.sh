#!/bin/bash
# r5: PMC counters of the expanding 1x1-conv GEMM (M=802816 N=256 K=64, cfg 8): HBM bytes and wave stall picture
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/r5y_p1" -o run -- python3 "$R/tools/gemm_conv1x1_bench.py" --cfgs 8 --only 802816,256,64 > "$R/gpurun_out/r5y_p1.log" 2>&1 || { tail -5 "$R/gpurun_out/r5y_p1.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES --kernel-trace -d "$R/gpurun_out/r5y_p2" -o run -- python3 "$R/tools/gemm_conv1x1_bench.py" --cfgs 8 --only 802816,256,64 > "$R/gpurun_out/r5y_p2.log" 2>&1 || { tail -5 "$R/gpurun_out/r5y_p2.log"; exit 1; }
cd "$R" && ls gpurun_out/r5y_p1 gpurun_out/r5y_p2 | head; find gpurun_out/r5y_p1 gpurun_out/r5y_p2 -name "*.csv" | head
