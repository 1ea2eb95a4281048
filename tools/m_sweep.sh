#!/bin/bash
# Bench step vs the wave encoder's sequence length (FEC_WAVE_M): bash tools/m_sweep.sh TAG M1 M2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
mkdir -p $R/gpurun_out/$TAG
cd $R
for M in "$@"; do
  FEC_WAVE_M=$M timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-host-inclusive --steps 30 > gpurun_out/$TAG/b$M.json 2> gpurun_out/$TAG/b$M.err || { tail -5 gpurun_out/$TAG/b$M.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/b$M.json')); print('M=$M', d['value'], d['ms_per_step'], d['kernels_ms_per_launch'])"
done
