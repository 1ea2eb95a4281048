#!/bin/bash
# The headline step's kernel times (rocprofv3 over tools/profile_step.py) and the step A/B tool's
# step time.   bash tools/gpu_enc_time.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-enct}
mkdir -p $OUT
cd $R && timeout -k 10 300 python3 -u tools/step_ab.py dedup=1 dedup=1 > $OUT/step.txt 2>&1 || { tail -20 $OUT/step.txt; exit 1; }
grep -v amdgpu.ids $OUT/step.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p -o run -- python3 $R/tools/profile_step.py --iters 200 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 $R/tools/kstats.py $(find $OUT/p -name '*kernel_stats.csv') > $OUT/stats.txt 2>&1
head -5 $OUT/stats.txt
