#!/bin/bash
# Copy kernel LDS row padding: parity tests, step A/B (FEC_COPY_ROW_PAD=0 vs default), LDS PMC pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-cpad}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_vr.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do for pad in 0 def; do
  if [ $pad = def ]; then unset FEC_COPY_ROW_PAD; else export FEC_COPY_ROW_PAD=$pad; fi
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-host-inclusive --no-extra-configs > $OUT/bench_$pad$i.json 2> $OUT/bench_$pad$i.err || { echo "bench failed"; tail -20 $OUT/bench_$pad$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_$pad$i.json').read().strip().splitlines()[-1]); print('pad $pad', d['value'], d['ms_per_step'], d['kernels_ms_per_launch'], d['kernels_ms_back_to_back'])"
done; done | tee $OUT/ab.txt
unset FEC_COPY_ROW_PAD
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --output-format csv -d $OUT/pmc -o pmc -- python3 $R/tools/profile_step.py --iters 3 > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
cd $R
timeout -k 10 60 python3 tools/pmc_summary.py $(find $OUT/pmc -name "*counter_collection.csv") > $OUT/pmc_summary.txt 2>&1 || true
grep -A5 "copy_fast\|encode_tile" $OUT/pmc_summary.txt | head -20
