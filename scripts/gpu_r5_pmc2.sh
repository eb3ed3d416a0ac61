#!/bin/bash
# r5: PMC roofline passes (counters + kernel trace only) over the final tree: ResNet-50 bs1024 and BERT-base;
# summarised on the box (tools/pmc_summary.py --last-step) and the raw CSVs dropped (gpurun_out is capped at 64 MiB)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/pmc6
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="FETCH_SIZE TCC_HIT_sum"
P3="WRITE_SIZE TCC_MISS_sum"
run() {  # name pass counters cmd...
  local name=$1 pass=$2 ctrs=$3; shift 3
  cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$R/gpurun_out/pmc6/$name/$pass" -o run -- "$@" > "$R/gpurun_out/pmc6/$name.$pass.log" 2>&1
  local rc=$?; cd "$R"; [ $rc -eq 0 ] || { echo "PMC_FAIL $name $pass rc=$rc"; tail -5 "$R/gpurun_out/pmc6/$name.$pass.log"; exit 1; }
  echo "PMC_OK $name $pass"
}
for p in 1 2 3; do
  eval C=\$P$p
  run resnet p$p "$C" python3 "$R/bench.py" --steps 2 --warmup 1 --batch 1024 --graph 0
  run bert p$p "$C" python3 "$R/tools/bench_bert.py" --steps 2 --warmup 1
done
python3 tools/pmc_summary.py gpurun_out/pmc6/resnet --top 25 --last-step > gpurun_out/r5_pmc_resnet_bs1024.txt 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc6/bert --top 20 --last-step > gpurun_out/r5_pmc_bert.txt 2>&1 || exit 1
rm -rf gpurun_out/pmc6
head -6 gpurun_out/r5_pmc_resnet_bs1024.txt
