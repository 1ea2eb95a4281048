"""Run bench.py's step (encode + plan + copy + recover) a few times without the extras, for
rocprofv3 kernel traces and PMC passes:  rocprofv3 --pmc ... -- python3 tools/profile_step.py"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import L, stream_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--packets", type=int, default=1_000_000)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--tbn", default="10,3,3")
ap.add_argument("--encode-path", default="auto")
args = ap.parse_args()
T, B, N = map(int, args.tbn.split(","))
torch.cuda.set_device(0)
P = args.packets
Pf = P + T
codec = Codec(L, T, B, N)
codec.set_encode_path(args.encode_path)
payload = fill_payload(0, Pf, L, 0x5EED)
er = torch.from_numpy(stream_pattern(Pf, 0)).cuda()
cw = torch.empty((Pf, codec.CW), dtype=torch.uint8, device="cuda")
wl = torch.empty(Pf, dtype=torch.int32, device="cuda")
out = torch.empty((P, L), dtype=torch.uint8, device="cuda")
ol = torch.empty(P, dtype=torch.int32, device="cuda")
for _ in range(args.iters):  # bench.py's step
    codec.encode(payload, out=cw, out_len=wl)
    codec.decode(cw, er, out=out, out_len=ol)
torch.cuda.synchronize()
print("ok", codec.counters(), codec.info())
