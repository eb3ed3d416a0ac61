#!/bin/bash
# Round-3 snapshot: canonical ResNet-50, BERT (bf16 / fp16), and one PMC pass of the zoo ResNet-50 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --variant canonical --batch 256 --steps 10 --warmup 4 > gpurun_out/r3_bench_canonical.log 2>&1 || { echo CANON_FAIL; tail -5 gpurun_out/r3_bench_canonical.log; exit 1; }
tail -1 gpurun_out/r3_bench_canonical.log
timeout -k 10 300 python3 tools/bench_bert.py --dtype bf16 > gpurun_out/r3_bench_bert_bf16.log 2>&1 || { echo BERT_FAIL; tail -5 gpurun_out/r3_bench_bert_bf16.log; exit 1; }
tail -1 gpurun_out/r3_bench_bert_bf16.log
timeout -k 10 300 python3 tools/bench_bert.py --dtype fp16 > gpurun_out/r3_bench_bert_fp16.log 2>&1 || { echo BERT16_FAIL; tail -5 gpurun_out/r3_bench_bert_fp16.log; exit 1; }
tail -1 gpurun_out/r3_bench_bert_fp16.log
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d "$R/gpurun_out/r3_pmc_halo" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --graph 0 > "$R/gpurun_out/r3_pmc_halo.log" 2>&1
rc=$?; cd "$R"; [ $rc -eq 0 ] && echo PMC_OK || { echo "PMC_FAIL rc=$rc"; tail -5 gpurun_out/r3_pmc_halo.log; exit 1; }
