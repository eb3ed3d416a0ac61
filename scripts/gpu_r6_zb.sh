#!/bin/bash
# r6zb: secondary benchmarks on the round-6 tree (BASELINE configs other than the headline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local n=$1; shift; timeout -k 10 400 "$@" > gpurun_out/r6zb_$n.json 2> gpurun_out/r6zb_$n.err || { echo "FAIL $n"; tail -5 gpurun_out/r6zb_$n.err; exit 1; }; echo "$n: $(tail -1 gpurun_out/r6zb_$n.json | cut -c1-230)"; }
run canonical python3 bench.py --variant canonical --batch 512 --steps 20 --warmup 5
run bs512 python3 bench.py --batch 512 --steps 20 --warmup 5
run bert python3 tools/bench_bert.py
run bert16 python3 tools/bench_bert.py --dtype fp16
run bertsd python3 tools/bench_bert_samediff.py
run lstm python3 tools/bench_lstm.py
run sdlstm python3 tools/bench_samediff_lstm.py
run lenet python3 tools/bench_lenet.py --device cuda --steps 100 --warmup 5
