#!/bin/bash
# Same-GPU PyTorch comparators + the framework's own numbers on the same box (zoo + canonical ResNet-50, LSTM)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
MIOPEN_FIND_MODE=2 timeout -k 10 400 python -u tools/bench_torch_comparators.py --model resnet50 --steps 10 --warmup 3 > gpurun_out/cmp_torch_resnet.log 2> gpurun_out/cmp_torch_resnet.err && tail -1 gpurun_out/cmp_torch_resnet.log &&
MIOPEN_FIND_MODE=2 timeout -k 10 300 python -u tools/bench_torch_comparators.py --model lstm --steps 3 --warmup 1 > gpurun_out/cmp_torch_lstm.log 2> gpurun_out/cmp_torch_lstm.err && tail -1 gpurun_out/cmp_torch_lstm.log &&
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nn_misc.py > gpurun_out/misc_tests.log 2>&1 && tail -2 gpurun_out/misc_tests.log &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_zoo.log 2>&1 && tail -1 gpurun_out/bench_zoo.log &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --variant canonical > gpurun_out/bench_canonical.log 2>&1 && tail -1 gpurun_out/bench_canonical.log &&
timeout -k 10 300 python -u tools/bench_lstm.py --steps 3 --warmup 1 > gpurun_out/bench_lstm.log 2>&1 && tail -1 gpurun_out/bench_lstm.log
