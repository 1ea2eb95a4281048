#!/bin/bash
# Round-6 final, part 1: the whole GPU suite, then the HBM traffic of the bench's kernels (the
# headline step over tools/profile_step.py, the type-2 relay chain over tools/swdf_bench.py):
# FETCH_SIZE and WRITE_SIZE in passes of their own, summarised with the source digest into
# gpurun_out/TAG/traffic.json (committed as profiles/r06/<TAG>_traffic.json before part 2, the bench).
#   bash tools/gpu_r06_final_pmc.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06final}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT/pmc
cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
i=0
for C in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc/step$i -o pmc -- python3 $R/tools/profile_step.py --iters 3 > $OUT/pmc/step$i.log 2>&1 || { echo "step pass $i failed"; tail -20 $OUT/pmc/step$i.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc/relay$i -o pmc -- python3 $R/tools/swdf_bench.py 2 > $OUT/pmc/relay$i.log 2>&1 || { echo "relay pass $i failed"; tail -20 $OUT/pmc/relay$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $(find $OUT/pmc -name '*counter_collection.csv') > $OUT/pmc_summary.txt
python3 $R/tools/pmc_traffic.py $OUT/traffic.json $TAG $OUT/pmc/step1 $OUT/pmc/step2 $OUT/pmc/relay1 $OUT/pmc/relay2 > $OUT/traffic.log 2>&1 || { tail -20 $OUT/traffic.log; exit 1; }
grep -E '"(fec_|traffic_bytes)' $OUT/traffic.json | head -30
