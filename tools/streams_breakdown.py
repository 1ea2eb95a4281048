"""Stream group call breakdown: host time inside encode / decode (launch returns) vs the whole call,
10 000 streams at (10,3,3).   python tools/streams_breakdown.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import StreamGroup, fill_payload  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402

torch.cuda.set_device(0)
NS, T, L = 10000, 10, 300
base = load_pattern("bin_erasure")[:360000]
grp = StreamGroup(L, T, 3, 3, NS)
ids = np.arange(NS, dtype=np.int32)
R = 60
pays = fill_payload(0, R * NS, L, 0xA11).view(R, NS, L)
ph = (36 * ids.astype(np.int64)) % base.size
ers = np.stack([base[(ph + r) % base.size] for r in range(R)]).astype(np.uint8)
cw = torch.empty((NS, grp.CW), dtype=torch.uint8, device="cuda")
wl = torch.empty(NS, dtype=torch.int32, device="cuda")
out = torch.empty((NS, L), dtype=torch.uint8, device="cuda")
ol = torch.empty(NS, dtype=torch.int32, device="cuda")
te, td = [], []
for r in range(10):
    grp.encode(ids, pays[r], out=cw, out_len=wl)
    grp.decode(ids, ers[r], cw, out=out, out_len=ol)
torch.cuda.synchronize()
t0 = time.perf_counter()
for r in range(10, R):
    a = time.perf_counter()
    grp.encode(ids, pays[r], out=cw, out_len=wl)
    b = time.perf_counter()
    grp.decode(ids, ers[r], cw, out=out, out_len=ol)
    c = time.perf_counter()
    te.append(b - a)
    td.append(c - b)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / (R - 10)
print(f"per call {dt * 1e6:.1f} us; host inside encode {np.median(te) * 1e6:.1f} us, inside decode "
      f"{np.median(td) * 1e6:.1f} us", flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, fn in (("encode", lambda r: grp.encode(ids, pays[r], out=cw, out_len=wl)),
                 ("decode", lambda r: grp.decode(ids, ers[r], cw, out=out, out_len=ol))):
    torch.cuda.synchronize()
    gpu = []
    for r in range(10, 30):
        e0.record()
        fn(r)
        e1.record()
        torch.cuda.synchronize()
        gpu.append(e0.elapsed_time(e1) * 1e3)
    print(f"{name}: event span {np.median(gpu):.1f} us (host launch included, synchronised per call)", flush=True)
