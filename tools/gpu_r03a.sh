#!/bin/bash
# Round 3, first GPU call: the --gpus launcher rehearsed on the 1-GPU box (2 ranks sharing the
# GPU over gloo), then the default N=1 bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r03a}
mkdir -p $OUT
cd $R
FEC_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_gloo2.json 2> $OUT/bench_gloo2.err || { echo "gloo2 bench failed"; tail -30 $OUT/bench_gloo2.err; exit 1; }
cat $OUT/bench_gloo2.json
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
