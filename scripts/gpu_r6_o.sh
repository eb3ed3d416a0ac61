#!/bin/bash
# r6o: BERT embedding kernels, step-kernel audits, BERT / LSTM / SameDiff GPU suites after the torch-op removal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_bert_embed.py tests/test_gpu_step_kernels.py tests/test_gpu_transformer.py tests/test_gpu_lstm.py tests/test_gpu_lstm_stack.py tests/test_gpu_lstm_graph.py tests/test_gpu_samediff.py > gpurun_out/r6o_tests.log 2>&1; rc=$?
grep -E "kernels,|torch:|FAIL|Error|passed|failed" gpurun_out/r6o_tests.log | head -40; exit $rc
