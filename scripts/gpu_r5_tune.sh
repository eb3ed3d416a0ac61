#!/bin/bash
# r5: record the gfx950 kernel-choice database (ops/tunedb.py) over the benchmark workloads, 8 timing repetitions
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out
export DL4J_AMD_TUNE_DB=off DL4J_AMD_TUNE_RECORD=$R/gpurun_out/tunedb_gfx950.json DL4J_AMD_TUNE_REPS=8
rm -f $DL4J_AMD_TUNE_RECORD
st() { local name=$1; shift; timeout -k 10 400 "$@" > gpurun_out/r5tune_$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/r5tune_$name.log; exit 1; }; echo "ok $name $(python3 -c "import json; print(sum(len(v) for v in json.load(open('$DL4J_AMD_TUNE_RECORD'))['tables'].values()))")"; }
st zoo1024 python3 bench.py --steps 3 --warmup 2
st zoo512 python3 bench.py --batch 512 --steps 3 --warmup 2
st canon512 python3 bench.py --variant canonical --batch 512 --steps 3 --warmup 2
st bert python3 tools/bench_bert.py --steps 3 --warmup 2
st bert16 python3 tools/bench_bert.py --dtype fp16 --steps 3 --warmup 2
st sdbert python3 tools/bench_bert_samediff.py --steps 3 --warmup 2
st lstm python3 tools/bench_lstm.py --steps 3 --warmup 2
st sdlstm python3 tools/bench_samediff_lstm.py --steps 3 --warmup 2
st lenet python3 tools/bench_lenet.py --steps 5 --warmup 2
