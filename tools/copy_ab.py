"""Decode copy kernels A/B in one process on the same buffers: bytes and lengths equal to the
LDS-tile copy ('fast'), then the kernel time alone and right after the encoder (as in the step).
  python tools/copy_ab.py fast generic [--tbn 10,3,3] [--packets 1000000]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import L, stream_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("paths", nargs="+")
ap.add_argument("--tbn", default="10,3,3")
ap.add_argument("--packets", type=int, default=1_000_000)
ap.add_argument("--rounds", type=int, default=5)
args = ap.parse_args()
torch.cuda.set_device(0)
TBN = tuple(int(x) for x in args.tbn.split(","))
P, T = args.packets, TBN[0]
Pf = P + T
codecs = {}
for p in args.paths:
    c = Codec(L, *TBN)
    c.set_copy_path(p)
    codecs[p] = c
payload = fill_payload(0, Pf, L, 0x5EED)
er = torch.from_numpy(stream_pattern(Pf, 0)).cuda()
c0 = Codec(L, *TBN)
c0.set_copy_path("fast")
cw, wl = c0.encode(payload)
ref_out, ref_len = c0.copy(cw, er)
out = torch.empty((P, L), dtype=torch.uint8, device="cuda")
ol = torch.empty(P, dtype=torch.int32, device="cuda")
for p, c in codecs.items():
    out.fill_(0xAB)
    ol.fill_(-7)
    c.copy(cw, er, out=out, out_len=ol)
    torch.cuda.synchronize()
    assert torch.equal(ol, ref_len), f"{p}: lengths differ"
    assert torch.equal(out, ref_out), f"{p}: bytes differ ({int((out != ref_out).any(1).sum())} rows)"
print(f"{TBN} {P} packets: all paths equal the LDS-tile copy", flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = {}
for rnd in range(args.rounds):
    for p, c in codecs.items():
        for mode in ["alone", "after_encode"]:
            t = []
            for _ in range(10):
                if mode == "after_encode":
                    c0.encode(payload, out=cw, out_len=wl)
                e0.record()
                c.copy(cw, er, out=out, out_len=ol)
                e1.record()
                torch.cuda.synchronize()
                t.append(e0.elapsed_time(e1) * 1e3)
            res.setdefault((p, mode), []).append(sorted(t)[5])
algo = (c0.CW + 1 + L) * P
for (p, mode), v in res.items():
    m = sorted(v)[len(v) // 2]
    print(f"{TBN} {p:6s} {mode:13s}: median {m:.1f} us = {algo / m / 1e3:.0f} GB/s "
          f"(rounds {', '.join(f'{x:.1f}' for x in v)})", flush=True)
