#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd "$R" && timeout -k 10 200 python -u -c "
import torch
from deeplearning4j_amd.models import ResNet50
from deeplearning4j_amd.nn.conf import DataType
from deeplearning4j_amd.ops import fallback
net = ResNet50(numLabels=1000, variant='canonical', dataType=DataType.BFLOAT16).init(device='cuda')
x = torch.rand(64, 3, 224, 224, device='cuda').contiguous(memory_format=torch.channels_last).bfloat16()
y = torch.zeros(64, 1000, device='cuda'); y[:, 3] = 1
fallback.reset(); net.fit([x], [y]); torch.cuda.synchronize()
print('fallbacks', fallback.summary())
" > gpurun_out/canon_fallbacks.log 2>&1; tail -3 gpurun_out/canon_fallbacks.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_canon" -o run -- python3 "$R/bench.py" --steps 3 --warmup 2 --variant canonical > "$R/gpurun_out/prof_canon.log" 2>&1
grep -q '"metric"' "$R/gpurun_out/prof_canon.log" && echo PROF_OK || { echo PROF_FAIL; exit 1; }
