#!/bin/bash
# Timing experiments on the wave encoder (FEC_WAVE_DBG bits, FEC_WAVE_M) -- encode kernel time only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for cfg in "0 0" "1 0" "2 0" "3 0" "0 96" "0 200"; do
  set -- $cfg
  FEC_WAVE_DBG=$1 FEC_WAVE_M=$2 timeout -k 10 120 python -u bench.py --encode-path wave --no-cpu-baseline --no-host-inclusive --steps 10 > /tmp/b.json 2>/tmp/b.err || { tail -5 /tmp/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('/tmp/b.json')); print('dbg=$1 M=$2', d['kernels_ms_per_launch']['fec_encode_kernel'])"
done
