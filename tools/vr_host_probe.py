"""Config 4 device calls: host submission time per call vs wall time per call (is a back-to-back
loop of fec_vr_encode_batch / fec_vr_decode_batch bound by the host or by the GPU?).
    python tools/vr_host_probe.py [calls]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import fill_payload  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.vr import VrPlan  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
torch.cuda.set_device(0)
P = 360000
v = VrPlan(load_pattern("bin_erasure"), P)
pl = fill_payload(0, v.sent, 300, 0x5EED)
frames = v.alloc_frames(zero=False)
out = torch.empty((P, 300), dtype=torch.uint8, device="cuda")
ol = torch.empty(P, dtype=torch.int32, device="cuda")
calls = [("encode", lambda: v.encode(pl, frames=frames)),
         ("decode", lambda: v.decode(frames[0], frames[2], out=out, out_len=ol)),
         ("encode+decode", lambda: (v.encode(pl, frames=frames), v.decode(frames[0], frames[2], out=out, out_len=ol)))]
for name, f in calls:
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(n):
            f()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{name}: submit {(t1 - t0) / n * 1e3:.3f} ms/call, wall {(t2 - t0) / n * 1e3:.3f} ms/call")
