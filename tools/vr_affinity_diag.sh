#!/bin/bash
# Config 4 plan timing with the process confined to a few CPUs vs the default placement.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-vraff}
mkdir -p $OUT
cd $R
C=fec_erasure_code_unit_test_relay_amd/csrc
python3 -c "
import sys; sys.path.insert(0,'.')
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern
load_pattern('bin_erasure').tofile('/tmp/bin_erasure.bin')" || exit 1
g++ -O2 -std=c++17 -pthread -I$C -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/vr_plan_bench.cpp $C/fec_vr.cpp $C/fec_host.cpp -o /tmp/vr_plan_bench -Lfec_erasure_code_unit_test_relay_amd -lfec_amd -Wl,-rpath,$R/fec_erasure_code_unit_test_relay_amd -L/opt/rocm/lib -lamdhip64 || exit 1
cat /proc/self/status | grep -i cpus_allowed_list
lscpu | grep -i "numa\|socket\|model name" | head -6
for i in 1 2 3; do
  for p in 0 1 2; do
    echo "FEC_VR_PIN=$p: $(FEC_VR_PIN=$p timeout 60 /tmp/vr_plan_bench /tmp/bin_erasure.bin 40 | cut -c1-60)"
  done
done | tee $OUT/aff.txt
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-host-inclusive --steps 20 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['configs']['config4_adaptive'])[:260])"
