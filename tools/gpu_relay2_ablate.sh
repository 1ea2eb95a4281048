#!/bin/bash
# Is the type-2 relay row scatter bound by its LDS byte writes?  Kernel times of the product build
# and of a -DFEC_RELAY2_ABLATE_WRITES build (one byte write per position instead of four; wrong
# output, timing only).   bash tools/gpu_relay2_ablate.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-relay2_ablate}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for V in product ablate; do
  if [ $V = ablate ]; then export FEC_AMD_LIB=$R/fec_erasure_code_unit_test_relay_amd/libfec_amd_abl.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$V -o run -- python3 $R/tools/swdf_bench.py 20 > $OUT/$V.log 2>&1 || { tail -20 $OUT/$V.log; exit 1; }
  python3 $R/tools/kstats.py $(find $OUT/$V -name '*kernel_stats.csv') > $OUT/${V}_stats.txt 2>&1
  echo "== $V"; grep -E "fast_relay2" $OUT/${V}_stats.txt
done
