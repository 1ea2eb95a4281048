set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05a
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/relay_prof.py 3 > $OUT/relay_prof.txt 2>&1 || { echo relay_prof failed; tail -20 $OUT/relay_prof.txt; exit 1; }
cat $OUT/relay_prof.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o relay -- python3 $R/tools/relay_prof.py 3 > $OUT/relay_prof_rocprof.txt 2>&1 || { echo rocprof failed; tail -20 $OUT/relay_prof_rocprof.txt; exit 1; }
KS=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cat "$KS" | cut -d, -f1-8
