#!/bin/bash
# Config 4 host-plan breakdown on the box, recovery beside the copy, graph vs eager step,
# encoder build variants.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-exp2}
mkdir -p $OUT
cd $R
C=fec_erasure_code_unit_test_relay_amd/csrc
python3 -c "
import sys; sys.path.insert(0,'.')
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern
load_pattern('bin_erasure').tofile('/tmp/bin_erasure.bin')"
g++ -O2 -std=c++17 -pthread -I$C -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/vr_plan_bench.cpp -o /tmp/vr_plan_bench -Lfec_erasure_code_unit_test_relay_amd -lfec_amd -Wl,-rpath,$R/fec_erasure_code_unit_test_relay_amd -L/opt/rocm/lib -lamdhip64
for t in 1 2 4 8; do echo "threads $t: $(FEC_VR_DEBUG=1 FEC_VR_THREADS=$t timeout 60 /tmp/vr_plan_bench /tmp/bin_erasure.bin 20 2>&1 | tail -3 | tr '\n' ' ')"; done | tee $OUT/vr_plan_threads.txt
timeout -k 10 200 python -u tools/lib_ab.py $C/../libfec_amd.so $C/../libfec_amd_b.so $C/../libfec_amd_c.so $C/../libfec_amd_d.so 2>&1 | tee $OUT/enc_variants.txt
timeout -k 10 200 python -u tools/step_env_ab.py "" "FEC_REC_BESIDE=1" 2>&1 | tee $OUT/beside_ab.txt
FEC_VR_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-inclusive > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d['configs']['config4_adaptive']))"
grep "vr control" $OUT/bench.err | tail -5
bash tools/graph_ab.sh exp2_graph 2>&1 | tee $OUT/graph_ab.txt
