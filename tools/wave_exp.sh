#!/bin/bash
# Timing experiments on the wave encoder alone (FEC_WAVE_DBG bits, FEC_WAVE_M).
#   bash tools/wave_exp.sh ["dbg M" ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
CFGS=("$@")
[ ${#CFGS[@]} -eq 0 ] && CFGS=("0 0" "1 0" "2 0" "3 0" "0 64" "0 96")
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  echo -n "dbg=$1 M=$2: "
  FEC_WAVE_DBG=$1 FEC_WAVE_M=$2 timeout -k 10 60 python -u tools/enc_time.py --path wave || exit 1
done
