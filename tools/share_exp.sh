#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for sh in 100 75 50 37 25; do
  echo "share=$sh"
  FEC_WAVE_SHARE=$sh timeout -k 10 120 python -u tools/pipe_exp.py 2>/dev/null | tail -2 || exit 1
done
