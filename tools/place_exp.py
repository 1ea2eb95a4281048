"""Encode time vs the codeword buffer's offset inside one allocation (HBM placement effects)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

torch.cuda.set_device(0)
P = 1_000_010
c = Codec(300, 10, 3, 3)
which = sys.argv[1] if len(sys.argv) > 1 else "cw"
big = torch.empty(P * 418 + (64 << 20), dtype=torch.uint8, device="cuda")
pbig = torch.empty(P * 300 + (64 << 20), dtype=torch.uint8, device="cuda")
wl = torch.empty(P, dtype=torch.int32, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
offs = [0, 4 << 10, 64 << 10, 256 << 10, 1 << 20, 2 << 20, 3 << 20, 4 << 20, 6 << 20, 8 << 20, 12 << 20, 16 << 20, 24 << 20, 32 << 20]
res = {}
for rnd in range(3):
    for o in offs:
        po = o if which == "payload" else 0
        co = o if which == "cw" else 0
        payload = pbig[po:po + P * 300].view(P, 300)
        if rnd == 0:
            fill_payload(0, P, 300, 0x5EED, out=payload)
        cw = big[co:co + P * 418].view(P, 418)
        c.encode(payload, out=cw, out_len=wl)
        e0.record()
        for _ in range(10):
            c.encode(payload, out=cw, out_len=wl)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(o, []).append(e0.elapsed_time(e1) * 100)
print(which, " ".join(f"{o >> 10}K:{sorted(v)[1]:.0f}" for o, v in res.items()))
