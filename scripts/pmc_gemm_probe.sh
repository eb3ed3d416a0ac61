#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p $R/gpurun_out/pmcg
export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/pmcg/p$i" -o run -- python3 $R/tools/gemm_probe.py --cfgs 4,2 --ks 64,768 --outs bf16 > "$R/gpurun_out/pmcg/p$i.log" 2>&1 || { echo PMC_FAIL $i; tail -5 $R/gpurun_out/pmcg/p$i.log; exit 1; }
  echo PMC_OK $i
done
