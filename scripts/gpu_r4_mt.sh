#!/bin/bash
# Graph-capture / in-process / RCCL GPU tests after the thread-local capture changes, then the stream-priority A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_inprocess_graphs.py tests/test_gpu_rccl.py tests/test_gpu_dist.py tests/test_gpu_samediff.py tests/test_gpu_lstm_graph.py -x -q -rs --timeout 150 --timeout-method thread > gpurun_out/r4_mt_tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4_mt_tests.log | head -30; tail -40 gpurun_out/r4_mt_tests.log; exit 1; }
tail -1 gpurun_out/r4_mt_tests.log
scripts/gpu_r4_prio.sh
