#!/bin/bash
# r5: in-kernel split-K fixup: GEMM tests, BERT bench fixup on/off, BERT kernel table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
j() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/r5aa_tests.log 2>&1 || { tail -30 gpurun_out/r5aa_tests.log; exit 1; }
tail -1 gpurun_out/r5aa_tests.log
for f in 1 0 1; do
  DL4J_AMD_GEMM_SPLITK_FIXUP=$f timeout -k 10 300 python3 tools/bench_bert.py > gpurun_out/r5aa_bert_$f.log 2>&1 || { tail -5 gpurun_out/r5aa_bert_$f.log; exit 1; }
  echo "bert fixup=$f $(j gpurun_out/r5aa_bert_$f.log)"
done
timeout -k 10 300 python3 tools/bench_bert_samediff.py > gpurun_out/r5aa_sdbert.log 2>&1 || { tail -5 gpurun_out/r5aa_sdbert.log; exit 1; }
echo "samediff bert $(j gpurun_out/r5aa_sdbert.log)"
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/r5aa_bprof" -o run -- python3 "$R/tools/bench_bert.py" --steps 4 --warmup 3 > "$R/gpurun_out/r5aa_bprof.log" 2>&1 || { tail -5 "$R/gpurun_out/r5aa_bprof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r5aa_bprof/run_results.db --top 30 > gpurun_out/r5aa_bert_step.txt && rm -rf gpurun_out/r5aa_bprof && head -16 gpurun_out/r5aa_bert_step.txt
