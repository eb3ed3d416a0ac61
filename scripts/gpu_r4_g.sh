#!/bin/bash
# Round-4: batched-load fused updater, SameDiff bias shadow (library GEMM candidate for SameDiff's linear ops):
# updater / SameDiff / transformer tests, BERT bf16 + fp16 (CG and SameDiff), ResNet, BERT step profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/r4g_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(grep -v amdgpu.ids "$R/gpurun_out/r4g_$name.log" | tail -1 | cut -c1-230)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
PT="python3 -u -m pytest -x -q --timeout 150 --timeout-method thread"
step t_upd 300 $PT tests/test_gpu_updaters_reference.py tests/test_gpu_updaters_gn.py tests/test_gpu_samediff.py tests/test_gpu_transformer.py
step b_bert 300 python3 tools/bench_bert.py --steps 10 --warmup 3
step b_bert_sd 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3
step b_bert16 300 python3 tools/bench_bert.py --steps 10 --warmup 3 --dtype fp16
step b_bert_sd16 300 python3 tools/bench_bert_samediff.py --steps 10 --warmup 3 --dtype fp16
step b_resnet 400 python3 bench.py --steps 30 --warmup 5
cd /tmp
step prof_bert 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4g_p_bert" -o run -- python3 "$R/tools/bench_bert.py" --steps 4 --warmup 3
cd "$R"
python3 tools/prof_laststep.py gpurun_out/r4g_p_bert/run_results.db --top 40 > gpurun_out/r4g_bert_step.txt 2>&1
rm -rf gpurun_out/r4g_p_bert; head -30 gpurun_out/r4g_bert_step.txt
