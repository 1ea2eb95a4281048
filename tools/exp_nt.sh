set -o pipefail
O=gpurun_out/nt; mkdir -p $O; : > $O/a.txt
for cfg in "" "FEC_COPY_NT=1" "FEC_TILE_DBG=8" "FEC_COPY_NT=1 FEC_TILE_DBG=8"; do
  env $cfg timeout -k 10 100 python -u tools/step_parts.py 2>&1 | grep "P=" | sed "s/^/[$cfg] /" >> $O/a.txt || exit 1
done
cat $O/a.txt
