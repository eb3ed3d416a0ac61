#!/bin/bash
# r6zf: end-of-round re-check after the late CPU-side ports (output-layer 3d labels, vocab, datavec): GPU suite,
# smoke(), one headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6zf_gpu_suite.log 2>&1; rc=$?; tail -2 gpurun_out/r6zf_gpu_suite.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r6zf_gpu_suite.log | head -20; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6zf_smoke.log 2>&1 || { tail -20 gpurun_out/r6zf_smoke.log; exit 1; }
tail -1 gpurun_out/r6zf_smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6zf_bench.json 2> gpurun_out/r6zf_bench.err || { tail -5 gpurun_out/r6zf_bench.err; exit 1; }
cut -c1-200 gpurun_out/r6zf_bench.json
