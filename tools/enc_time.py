"""Encode kernel alone: average time per launch over 1M packets (10,3,3), no concurrent kernels.
  python tools/enc_time.py [--path wave] [--iters 20] [--tbn 10,3,3] [--packets 1000010]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--path", default="auto")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--tbn", default="10,3,3")
ap.add_argument("--packets", type=int, default=1_000_010)
args = ap.parse_args()
T, B, N = map(int, args.tbn.split(","))
torch.cuda.set_device(0)
c = Codec(300, T, B, N)
c.set_encode_path(args.path)
P = args.packets
payload = fill_payload(0, P, 300, 0x5EED)
cw = torch.empty((P, c.CW), dtype=torch.uint8, device="cuda")
wl = torch.empty(P, dtype=torch.int32, device="cuda")
for _ in range(3):
    c.encode(payload, out=cw, out_len=wl)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(args.iters):
    c.encode(payload, out=cw, out_len=wl)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / args.iters
print(f"{args.path} {args.tbn} P={P}: {us:.1f} us/launch, {(300 + c.CW) * P / us / 1e3:.0f} GB/s algorithmic",
      flush=True)
