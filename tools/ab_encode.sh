set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for p in fast stream; do
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_$p -o run -- python3 $R/tools/profile_step.py --iters 5 --encode-path $p > $R/gpurun_out/ab_$p.log 2>&1
done
