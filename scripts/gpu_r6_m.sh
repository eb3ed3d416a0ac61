#!/bin/bash
# r6m: step-kernel audits (ResNet-50, BERT, LSTM char-LM)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_step_kernels.py > gpurun_out/r6m_audit.log 2>&1; rc=$?
grep -E "kernels,|torch:|PASS|FAIL|Error" gpurun_out/r6m_audit.log | head -60; exit $rc
