#!/bin/bash
# Round-3 PMC tables (MFMA busy / LDS conflicts) of the last step: final ResNet-50 tree and BERT-base (bf16).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d "$R/gpurun_out/r3c_pmc_bert" -o run -- python3 "$R/tools/bench_bert.py" --steps 2 --warmup 3 --graph 0 > "$R/gpurun_out/r3c_pmc_bert.log" 2>&1
rc=$?; cd "$R"; [ $rc -eq 0 ] || { echo "PMC_FAIL rc=$rc"; tail -5 gpurun_out/r3c_pmc_bert.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r3c_pmc_bert --last-step --top 25 > gpurun_out/r3c_pmc_bert_table.txt && cat gpurun_out/r3c_pmc_bert_table.txt
rm -rf gpurun_out/r3c_pmc_bert/*.db
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d "$R/gpurun_out/r3c_pmc_zoo" -o run -- python3 "$R/bench.py" --steps 2 --warmup 3 --graph 0 > "$R/gpurun_out/r3c_pmc_zoo.log" 2>&1
rc=$?; cd "$R"; [ $rc -eq 0 ] || { echo "PMC_FAIL rc=$rc"; tail -5 gpurun_out/r3c_pmc_zoo.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r3c_pmc_zoo --last-step --top 30 > gpurun_out/r3c_pmc_zoo_table.txt && head -12 gpurun_out/r3c_pmc_zoo_table.txt
