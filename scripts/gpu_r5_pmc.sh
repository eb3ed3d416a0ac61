#!/bin/bash
# rocprofv3 PMC counter passes (one run per pass: counters + kernel trace only, no runtime/sys tracing) over the
# ResNet-50 bench, BERT and LSTM benches. Summaries: python tools/pmc_summary.py gpurun_out/pmc5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc5
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="FETCH_SIZE TCC_HIT_sum"
P3="WRITE_SIZE TCC_MISS_sum"
run() {  # name pass counters cmd...
  local name=$1 pass=$2 ctrs=$3; shift 3
  cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$R/gpurun_out/pmc5/$name/$pass" -o run -- "$@" > "$R/gpurun_out/pmc5/$name.$pass.log" 2>&1
  local rc=$?; cd "$R"; [ $rc -eq 0 ] || { echo "PMC_FAIL $name $pass rc=$rc"; tail -5 "$R/gpurun_out/pmc5/$name.$pass.log"; exit 1; }
  echo "PMC_OK $name $pass"
}
for p in ${PMC_PASSES:-1 2 3}; do
  eval C=\$P$p
  run resnet p$p "$C" python3 "$R/bench.py" --steps 2 --warmup 1 --batch 1024 --graph 0
  run bert p$p "$C" python3 "$R/tools/bench_bert.py" --steps 2 --warmup 1
  [ -n "$PMC_LSTM" ] && run lstm p$p "$C" python3 "$R/tools/bench_lstm.py" --steps 1 --warmup 1 --length 200
done
