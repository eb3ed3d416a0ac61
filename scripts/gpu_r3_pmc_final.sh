#!/bin/bash
# Round-3 steady-state PMC table of the ResNet-50 bench (one pass: MFMA busy / LDS counters), last step only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d "$R/gpurun_out/r3_pmc_final" -o run -- python3 "$R/bench.py" --steps 2 --warmup 3 --graph 0 > "$R/gpurun_out/r3_pmc_final.log" 2>&1
rc=$?; cd "$R"; [ $rc -eq 0 ] || { echo "PMC_FAIL rc=$rc"; tail -5 gpurun_out/r3_pmc_final.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r3_pmc_final --last-step --top 30 > gpurun_out/r3_pmc_final_table.txt && cat gpurun_out/r3_pmc_final_table.txt
