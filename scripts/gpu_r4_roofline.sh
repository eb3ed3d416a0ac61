#!/bin/bash
# Round-4 per-kernel roofline of ONE steady-state training step (last step): three rocprofv3 counter passes
# (P1 MFMA/LDS, P2 FETCH_SIZE + L2 hits, P3 WRITE_SIZE + L2 misses), each its own run with --kernel-trace only.
# Usage: scripts/gpu_r4_roofline.sh <tag> <python args...>   (e.g. resnet bench.py --steps 2 --warmup 3 --graph 0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$GRAFT_REPO_ROOT"
TAG=$1; shift
mkdir -p gpurun_out/roof
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="FETCH_SIZE TCC_HIT_sum"
P3="WRITE_SIZE TCC_MISS_sum"
for p in 1 2 3; do
  eval C=\$P$p
  cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/roof/$TAG/p$p" -o run -- python3 "$R/$@" > "$R/gpurun_out/roof/$TAG.p$p.log" 2>&1
  rc=$?; cd "$R"; [ $rc -eq 0 ] || { echo "PMC_FAIL $TAG p$p rc=$rc"; tail -5 "gpurun_out/roof/$TAG.p$p.log"; exit 1; }
  rm -f gpurun_out/roof/$TAG/p$p/*.db
  echo "PMC_OK $TAG p$p"
done
python3 tools/pmc_summary.py gpurun_out/roof/$TAG --last-step --top 40 > gpurun_out/roof/${TAG}_table.txt && cat gpurun_out/roof/${TAG}_table.txt && rm -rf gpurun_out/roof/$TAG
