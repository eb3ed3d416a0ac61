#!/bin/bash
# Round-4: stem weight-gradient kernel (two-round dy look-ahead, 3 workgroups/CU), BN+pool backward with batched x
# loads, vectorized GELU after library GEMMs. Tests, ResNet / BERT benches, ResNet and SameDiff-BERT step profiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4h_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4h_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step t_bn 300 $PT tests/test_gpu_bnpool.py tests/test_gpu_gemm.py -k "bn_pool or stem or library"
step b_resnet 400 python3 bench.py --steps 30 --warmup 5
step b_bert 300 python3 tools/bench_bert.py --steps 10 --warmup 3
prof() {   # prof <name> <cmd...>
  local name=$1; shift
  cd /tmp
  step "prof_$name" 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4h_p_$name" -o run -- "$@"
  cd "$R"
  python3 tools/prof_laststep.py "gpurun_out/r4h_p_$name/run_results.db" --top 40 > "gpurun_out/r4h_${name}_step.txt" 2>&1
  python3 tools/prof_steplist.py "gpurun_out/r4h_p_$name/run_results.db" > "gpurun_out/r4h_${name}_steplist.txt" 2>&1
  rm -rf "gpurun_out/r4h_p_$name"; head -24 "gpurun_out/r4h_${name}_step.txt"
}
prof resnet python3 "$R/bench.py" --steps 4 --warmup 3
prof sdbert python3 "$R/tools/bench_bert_samediff.py" --steps 4 --warmup 3
