"""Dump config 4's decode-copy inputs for tools/ubench/vr_copy_real.hip: per packet the copy's
geometry word (k | n << 8 | fate << 16, as fec_vr_geo_kernel; the slow flag left 0) and the cur
rows' offsets of the compact layout.   python tools/vr_dump.py [out_dir]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.vr import VrPlan  # noqa: E402
from fec_erasure_code_unit_test_relay_amd._lib import lib  # noqa: E402,F401

out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tools", "ubench", "data")
os.makedirs(out, exist_ok=True)
P = 360000
v = VrPlan(load_pattern("bin_erasure"), P)
# decoder instance geometry: k = T - N + 1, n = k + B
T, B, N = v.decoders[:, 0], v.decoders[:, 1], v.decoders[:, 2]
k = T - N + 1
n = k + B
f = v.fate.astype(np.uint32)
j = v.fate_decoder
geo = f << 16
rec = f == 1
geo[rec] |= (k[j[rec]] | (n[j[rec]] << 8)).astype(np.uint32)
co, _ = v.row_offsets()
geo.astype(np.uint32).tofile(os.path.join(out, "vr_geo.bin"))
co.astype(np.int64).tofile(os.path.join(out, "vr_curoff.bin"))
print(P, v.sent, int(co[-1]), np.bincount(f, minlength=4))
