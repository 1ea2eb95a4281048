#!/bin/bash
# Device assembly of one source file (gfx950) with its kernel resource metadata:
#   bash tools/isa.sh fec_copy_fast.hip > /tmp/copy_fast.s
cd "$(dirname "$0")/../fec_erasure_code_unit_test_relay_amd/csrc" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -I. --cuda-device-only -S -o - "$@"
