#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3_halo_kt" -o run -- python3 "$R/tools/wrw_halo_probe.py" --variant 1 --splits 256 --reps 3 > "$R/gpurun_out/r3_halo_kt.log" 2>&1 || { echo kt fail; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/r3_halo_pmc1" -o run -- python3 "$R/tools/wrw_halo_probe.py" --variant 1 --splits 256 --reps 2 > "$R/gpurun_out/r3_halo_pmc1.log" 2>&1 || { echo pmc1 fail; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace --output-format csv -d "$R/gpurun_out/r3_halo_pmc2" -o run -- python3 "$R/tools/wrw_halo_probe.py" --variant 1 --splits 256 --reps 2 > "$R/gpurun_out/r3_halo_pmc2.log" 2>&1 || { echo pmc2 fail; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d "$R/gpurun_out/r3_halo_pmc3" -o run -- python3 "$R/tools/wrw_halo_probe.py" --variant 1 --splits 256 --reps 2 > "$R/gpurun_out/r3_halo_pmc3.log" 2>&1 || { echo pmc3 fail; exit 1; }
echo done
