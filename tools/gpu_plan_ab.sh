#!/bin/bash
# Config 4 host plan on the box host: variants interleaved (tools/vr_plan_ab.py), then the control
# loop's cycle split and iteration classes (vr_plan_bench_prof, a -DFEC_VR_PROFILE build of
# fec_vr.cpp) with the default stretches and with FEC_VR_FB_STOP.   bash tools/gpu_plan_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-plan_ab}
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u tools/vr_plan_ab.py 6 > $OUT/plan_ab.txt 2>&1 || { tail -20 $OUT/plan_ab.txt; exit 1; }
cat $OUT/plan_ab.txt
python3 -c "from fec_erasure_code_unit_test_relay_amd.streams import load_pattern; load_pattern('bin_erasure').tofile('$OUT/pat.bin')"
CPUS=$(python3 -c "import sys; sys.path.insert(0, '.'); from bench import quiet_cpu_group; g = quiet_cpu_group(); print(f'{g[0]}-{g[-1]}' if g else '')")
for V in X FEC_VR_FB_STOP; do
  if [ -n "$CPUS" ]; then
    env $V=1 FEC_VR_DEBUG=1 timeout -k 10 60 taskset -c $CPUS ./tools/ubench/vr_plan_bench_prof $OUT/pat.bin 6 > $OUT/prof_$V.txt 2>&1 || { tail -5 $OUT/prof_$V.txt; exit 1; }
  else
    env $V=1 FEC_VR_DEBUG=1 timeout -k 10 60 ./tools/ubench/vr_plan_bench_prof $OUT/pat.bin 6 > $OUT/prof_$V.txt 2>&1 || { tail -5 $OUT/prof_$V.txt; exit 1; }
  fi
  echo "== $V"; grep -E "Mcycles|loop thread|drops|plan" $OUT/prof_$V.txt | tail -4
done
rm -f $OUT/pat.bin
