#!/bin/bash
# Round verification on the current sources, then the side-stream CU-mask A/B.
set -o pipefail
bash tools/gpu_round.sh r03z || exit 1
bash tools/side_cus_ab.sh r03z_side 2>&1 | tee gpurun_out/r03z/side_cus_ab.txt
