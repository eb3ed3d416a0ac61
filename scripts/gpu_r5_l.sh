#!/bin/bash
# r5: multi-GPU paths at world 1 — in-process ParallelWrapper (graphs) vs the eager headline, 1-rank RCCL process group
# with forced collectives (timing + kernel trace: bucket all-reduces overlapping backward)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
val() { tail -1 "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('parallelism'), d['config'].get('hip_graph'))"; }
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5l_eager.log 2>&1 || { tail -20 gpurun_out/r5l_eager.log; exit 1; }
echo "eager headline: $(val gpurun_out/r5l_eager.log)" | tee gpurun_out/r5l.log
timeout -k 10 400 python3 bench.py --inprocess 1 --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5l_inproc.log 2>&1 || { tail -20 gpurun_out/r5l_inproc.log; exit 1; }
echo "in-process world 1: $(val gpurun_out/r5l_inproc.log)" | tee -a gpurun_out/r5l.log
DL4J_AMD_FORCE_COLLECTIVES=1 timeout -k 10 400 python3 bench.py --inprocess 1 --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5l_inproc_f.log 2>&1 || { tail -20 gpurun_out/r5l_inproc_f.log; exit 1; }
echo "in-process world 1 forced collectives: $(val gpurun_out/r5l_inproc_f.log)" | tee -a gpurun_out/r5l.log
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 DL4J_AMD_FORCE_COLLECTIVES=1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5l_pg.log 2>&1 || { tail -20 gpurun_out/r5l_pg.log; exit 1; }
echo "process group world 1 forced collectives: $(val gpurun_out/r5l_pg.log)" | tee -a gpurun_out/r5l.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/r5l_prof" -o run -- python3 "$R/bench.py" --steps 3 --warmup 4 > "$R/gpurun_out/r5l_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r5l_prof.log"; exit 1; }
cd "$R" && python3 tools/overlap_report.py gpurun_out/r5l_prof/run_results.db > gpurun_out/r5l_overlap.txt && rm -rf gpurun_out/r5l_prof && tail -25 gpurun_out/r5l_overlap.txt
