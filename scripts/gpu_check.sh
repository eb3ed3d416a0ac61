#!/bin/bash
# One GPU session: build, smoke, GPU tests, short bench, kernel-trace profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
echo SMOKE_OK
timeout -k 10 900 python -m pytest tests/ -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
  echo PROF_OK
fi
