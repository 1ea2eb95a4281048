#!/bin/bash
# wave encoder A/B by environment: bash tools/pad_exp.sh VAR "v1 v2" [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
VAR=${1:-FEC_WAVE_PAD}; VALS=${2:-"0 1"}; ROUNDS=${3:-3}
for r in $(seq $ROUNDS); do
  for v in $VALS; do
    echo -n "$VAR=$v: "
    env $VAR=$v timeout -k 10 60 python -u tools/enc_time.py --path wave 2>/dev/null || exit 1
  done
done
