#!/bin/bash
# Round-4: per-step kernel tables of the ResNet-50 and BERT benches, BERT fp16 (CG and SameDiff), and the per-shape
# conv table at bs512. A crash / abort / time limit ends the run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4e_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4e_$name.log" | tail -1 | cut -c1-220)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
prof() {   # prof <name> <cmd...>: kernel trace of a short run, last-step table
  local name=$1; shift
  cd /tmp
  step "prof_$name" 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4e_p_$name" -o run -- "$@"
  cd "$R"
  python3 tools/prof_laststep.py "gpurun_out/r4e_p_$name/run_results.db" --top 40 > "gpurun_out/r4e_${name}_step.txt" 2>&1
  python3 tools/prof_steplist.py "gpurun_out/r4e_p_$name/run_results.db" > "gpurun_out/r4e_${name}_steplist.txt" 2>&1
  rm -rf "gpurun_out/r4e_p_$name"; head -14 "gpurun_out/r4e_${name}_step.txt"
}
prof resnet python3 "$R/bench.py" --steps 4 --warmup 3
step choices 300 python3 tools/conv_choices.py --batch 512
grep -v amdgpu.ids gpurun_out/r4e_choices.log | head -80
prof bert python3 "$R/tools/bench_bert.py" --steps 4 --warmup 3
step bert_fp16 300 python3 tools/bench_bert.py --steps 10 --warmup 3 --dtype fp16
step bert_sd_fp16 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3 --dtype fp16
step conv_shapes 600 python3 -u tools/conv_bench.py --batch 512 --reps 10
grep -v amdgpu.ids gpurun_out/r4e_conv_shapes.log | head -70
