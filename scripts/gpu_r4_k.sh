#!/bin/bash
# Round-4: SameDiff BERT fp16 vs bf16 (step kernel tables), CG BERT fp16.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4k_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4k_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
step b_bert16 300 python3 tools/bench_bert.py --steps 10 --warmup 3 --dtype fp16
prof() {   # prof <name> <cmd...>
  local name=$1; shift
  cd /tmp
  step "prof_$name" 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4k_p_$name" -o run -- "$@"
  cd "$R"
  python3 tools/prof_laststep.py "gpurun_out/r4k_p_$name/run_results.db" --top 40 > "gpurun_out/r4k_${name}_step.txt" 2>&1
  python3 tools/prof_steplist.py "gpurun_out/r4k_p_$name/run_results.db" > "gpurun_out/r4k_${name}_steplist.txt" 2>&1
  rm -rf "gpurun_out/r4k_p_$name"; head -30 "gpurun_out/r4k_${name}_step.txt"
}
prof sd16 python3 "$R/tools/bench_bert_samediff.py" --steps 4 --warmup 3 --dtype fp16
prof sd python3 "$R/tools/bench_bert_samediff.py" --steps 4 --warmup 3
