#!/bin/bash
# Tile encoder LDS diagnosis: bank-conflict / LDS counters with each phase ablated (FEC_TILE_DBG:
# 0 full, 1 no parity products, 2 no codeword words, 4 no output stores), one rocprofv3 pass each.
# The ablations exist in the runtime-L kernel only: L = 296 (not the L = 300 specialisation).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-tile_lds}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for d in 0 1 2 4 7; do
  FEC_TILE_DBG=$d timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d $OUT/d$d -o pmc -- python3 $R/tools/enc_time.py --iters 3 --reps 1 --L ${FEC_DIAG_L:-296} > $OUT/d$d.log 2>&1 || { echo "pass $d failed"; tail -20 $OUT/d$d.log; exit 1; }
  echo "== FEC_TILE_DBG=$d"
  python3 $R/tools/pmc_summary.py $(find $OUT/d$d -name '*counter_collection.csv') | grep -A6 encode_tile
done
