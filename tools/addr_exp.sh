#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for sh in 0 0 0 0 1 2 3 4 5 6 7 8 16 32 64 100; do
  echo -n "shift=$sh: "
  ENC_SHIFT_MB=$sh timeout -k 10 60 python -u tools/enc_time.py --path wave --reps 5 2>/dev/null || exit 1
done
