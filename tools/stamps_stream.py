"""Phase cycles of the streaming encode kernel (sums per workgroup over its tiles)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import L  # noqa: E402
from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload, lib  # noqa: E402

torch.cuda.set_device(0)
P = 1_000_010
codec = Codec(L, 10, 3, 3)
codec.set_encode_path("stream")
print(codec.info())
payload = fill_payload(0, P, L, 0x5EED)
cw, wl = codec.encode(payload)
st = torch.zeros(65536 * 8, dtype=torch.int64, device="cuda")
for it in range(3):
    st.zero_()
    lib().fec_debug_stamps(codec._h, 0, ctypes.c_void_p(st.data_ptr()))
    codec.encode(payload, out=cw, out_len=wl)
    torch.cuda.synchronize()
    lib().fec_debug_stamps(codec._h, 0, None)
s = st.cpu().numpy().reshape(-1, 8)
s = s[s[:, 7] > 0].astype(np.float64)
tiles = s[:, 7]
print(f"workgroups {len(s)}, tiles per workgroup {tiles.min():.0f}..{tiles.max():.0f}")
names = ["prologue", "load+prefetch", "transpose", "parity", "interleave", "store+carry"]
tot = s[:, 6]
print(f"workgroup life: mean {tot.mean():.0f} cycles, per tile {np.mean(tot / tiles):.0f}")
for k, nm in enumerate(names):
    per_tile = s[:, k] / (tiles if k else 1)
    print(f"  {nm:14s} mean {per_tile.mean():9.0f} cycles{' per tile' if k else ''}")
