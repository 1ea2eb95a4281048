"""Encode kernel alone: average time per launch over 1M packets (10,3,3), no concurrent kernels.
  python tools/enc_time.py [--path tile] [--iters 20] [--tbn 10,3,3] [--packets 1000010]"""
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
ap.add_argument("--reps", type=int, default=7)
ap.add_argument("--ab", default="", help="comma-separated FEC_WAVE_DBG values (or VAR=value) timed in one process")
ap.add_argument("--tbn", default="10,3,3")
ap.add_argument("--packets", type=int, default=1_000_010)
ap.add_argument("--L", type=int, default=300, help="payload size (300: the kernels specialised on L = 300)")
args = ap.parse_args()
T, B, N = map(int, args.tbn.split(","))
torch.cuda.set_device(0)
c = Codec(args.L, T, B, N)
c.set_encode_path(args.path)
P = args.packets
ap2 = os.environ.get("ENC_SHIFT_MB")
if ap2:  # experiment: shift the allocations by a dummy block
    _dummy = torch.empty(int(float(ap2) * 2**20), dtype=torch.uint8, device="cuda")
payload = fill_payload(0, P, args.L, 0x5EED)
cw = torch.empty((P, c.CW), dtype=torch.uint8, device="cuda")
wl = torch.empty(P, dtype=torch.int32, device="cuda")
for _ in range(3):
    c.encode(payload, out=cw, out_len=wl)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
if args.ab:  # in-process A/B over FEC_WAVE_DBG values (same buffers, alternating batches)
    res = {v: [] for v in args.ab.split(",")}
    for _ in range(args.reps):
        for v in res:
            var, val = v.split("=") if "=" in v else ("FEC_WAVE_DBG", v)
            os.environ[var] = val
            c.encode(payload, out=cw, out_len=wl)
            e0.record()
            for _ in range(args.iters):
                c.encode(payload, out=cw, out_len=wl)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) * 1e3 / args.iters)
    print("  ".join(f"{v}: {sorted(x)[len(x) // 2]:.1f} us" for v, x in res.items()), flush=True)
    sys.exit(0)
samples = []
for _ in range(args.reps):  # median of several timed batches (box-to-box and clock noise)
    e0.record()
    for _ in range(args.iters):
        c.encode(payload, out=cw, out_len=wl)
    e1.record()
    torch.cuda.synchronize()
    samples.append(e0.elapsed_time(e1) * 1e3 / args.iters)
us = sorted(samples)[len(samples) // 2]
print(f"payload@{payload.data_ptr():#x} cw@{cw.data_ptr():#x} "
      f"{args.path} {args.tbn} P={P}: {us:.1f} us/launch, {(args.L + c.CW) * P / us / 1e3:.0f} GB/s algorithmic",
      flush=True)
