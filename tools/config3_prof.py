"""BASELINE config 3 alone (bench.py extra_configs): device-resident decode at (10,5,2) of 360 000
packets on bin/erasure.bin replayed from packet 0, `iters` timed decodes after 3 warm-ups, for a
rocprofv3 kernel trace of its launch chain:
    rocprofv3 --kernel-trace --stats -- python3 tools/config3_prof.py [iters]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
L, P = 300, 360000
torch.cuda.set_device(0)
pat = load_pattern("bin_erasure")
c = Codec(L, 10, 5, 2)
payload = fill_payload(0, P + 10, L, 0x5EED)
cw, _ = c.encode(payload)
er = torch.from_numpy(pat[:P + 10].copy()).cuda()
out = torch.empty((P, L), dtype=torch.uint8, device="cuda")
ol = torch.empty(P, dtype=torch.int32, device="cuda")
c.workspace(P + 10)
for _ in range(3):
    c.decode(cw, er, out=out, out_len=ol)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(iters):
    c.decode(cw, er, out=out, out_len=ol)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / iters
lost = int((ol == 0).sum())
print(f"config 3 decode: {dt * 1e3:.4f} ms per 360000 packets, lost {lost} (expected 565)", flush=True)
