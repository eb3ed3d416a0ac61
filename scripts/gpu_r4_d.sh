#!/bin/bash
# Round-4 after the stack/sink/lib changes: full GPU suite, then per-step kernel tables of the LSTM (stacked), BERT
# (CG graph) and ResNet-50 benches, and the per-shape conv table at bs512. A crash / abort / time limit ends the run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4d_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4d_$name.log" | tail -1 | cut -c1-220)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
step suite 900 python3 -u -m pytest tests -q -m gpu -rs --maxfail 5 --timeout 150 --timeout-method thread
grep -E "^FAILED|^ERROR" gpurun_out/r4d_suite.log | head -20
prof() {   # prof <name> <cmd...>: kernel trace of a short run, last-step table
  local name=$1; shift
  cd /tmp
  step "prof_$name" 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4d_p_$name" -o run -- "$@"
  cd "$R"
  python3 tools/prof_laststep.py "gpurun_out/r4d_p_$name/run_results.db" --top 40 > "gpurun_out/r4d_${name}_step.txt" 2>&1
  rm -rf "gpurun_out/r4d_p_$name"; head -14 "gpurun_out/r4d_${name}_step.txt"
}
prof lstm python3 "$R/tools/bench_lstm.py" --steps 4 --warmup 2
prof bert python3 "$R/tools/bench_bert.py" --steps 4 --warmup 3
prof resnet python3 "$R/bench.py" --steps 4 --warmup 3
step conv_shapes 600 python3 -u tools/conv_bench.py --batch 512 --reps 10
grep -v amdgpu.ids gpurun_out/r4d_conv_shapes.log | head -70
