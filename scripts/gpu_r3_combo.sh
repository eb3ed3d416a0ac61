#!/bin/bash
# Full GPU suite, headline bench, then the phase-split checks (canonical bench, zoo step list), then the PMC table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 480 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3_suite_reentry.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r3_suite_reentry.log | head -30; tail -5 gpurun_out/r3_suite_reentry.log; exit 1; }
tail -1 gpurun_out/r3_suite_reentry.log
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_reentry.log 2>&1 || { tail -20 gpurun_out/r3_bench_reentry.log; exit 1; }
tail -1 gpurun_out/r3_bench_reentry.log
timeout -k 10 400 python3 bench.py --variant canonical --steps 10 --warmup 4 > gpurun_out/r3_bench_canonical_phase.log 2>&1 || { tail -20 gpurun_out/r3_bench_canonical_phase.log; exit 1; }
tail -1 gpurun_out/r3_bench_canonical_phase.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r3_prof_zoo" -o run -- python3 "$R/bench.py" --steps 4 --warmup 3 > "$R/gpurun_out/r3_prof_zoo.log" 2>&1 || { tail -5 "$R/gpurun_out/r3_prof_zoo.log"; exit 1; }
cd "$R" && python3 tools/prof_steplist.py gpurun_out/r3_prof_zoo/run_results.db > gpurun_out/r3_zoo_steplist.txt && python3 tools/prof_laststep.py gpurun_out/r3_prof_zoo/run_results.db --top 40 > gpurun_out/r3_zoo_step.txt && rm -f gpurun_out/r3_prof_zoo/run_results.db && tail -1 gpurun_out/r3_zoo_steplist.txt && head -12 gpurun_out/r3_zoo_step.txt
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d "$R/gpurun_out/r3_pmc_final" -o run -- python3 "$R/bench.py" --steps 2 --warmup 3 --graph 0 > "$R/gpurun_out/r3_pmc_final.log" 2>&1
rc=$?; cd "$R"; [ $rc -eq 0 ] || { echo "PMC_FAIL rc=$rc"; tail -5 gpurun_out/r3_pmc_final.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r3_pmc_final --last-step --top 30 > gpurun_out/r3_pmc_final_table.txt && cat gpurun_out/r3_pmc_final_table.txt
