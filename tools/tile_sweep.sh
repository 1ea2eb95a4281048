# Kernel times of the step at several tile caps (rocprofv3 kernel trace per setting).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for t in 64 32 16; do
  FEC_ENCODE_TILE=$t FEC_COPY_TILE=$t timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tile$t -o run -- python3 $R/tools/profile_step.py --iters 5 > $R/gpurun_out/tile$t.log 2>&1
done
