#!/bin/bash
# r5: smoke score on one box, session-start code vs current code, twice each (is the score change code or box?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  (cd _smoke_old && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()") > gpurun_out/r5am_old$r.log 2>&1 || { tail -5 gpurun_out/r5am_old$r.log; exit 1; }
  echo "old$r $(tail -1 gpurun_out/r5am_old$r.log | cut -c1-60)"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5am_new$r.log 2>&1 || { tail -5 gpurun_out/r5am_new$r.log; exit 1; }
  echo "new$r $(tail -1 gpurun_out/r5am_new$r.log | cut -c1-60)"
done
