#!/bin/bash
# r5: one-step kernel table of the ResNet-50 bench (bs1024) and of BERT (in-tree GEMMs only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/r5i_prof" -o run -- python3 "$R/bench.py" --steps 3 --warmup 4 > "$R/gpurun_out/r5i_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r5i_prof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r5i_prof/run_results.db --top 45 > gpurun_out/r5i_resnet_step.txt && rm -rf gpurun_out/r5i_prof && head -50 gpurun_out/r5i_resnet_step.txt
cd /tmp && DL4J_AMD_GEMM_LIB=0 timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/r5i_bprof" -o run -- python3 "$R/tools/bench_bert.py" --steps 4 --warmup 3 > "$R/gpurun_out/r5i_bprof.log" 2>&1 || { tail -5 "$R/gpurun_out/r5i_bprof.log"; exit 1; }
cd "$R" && python3 tools/prof_laststep.py gpurun_out/r5i_bprof/run_results.db --top 30 > gpurun_out/r5i_bert_step.txt && rm -rf gpurun_out/r5i_bprof && head -34 gpurun_out/r5i_bert_step.txt
