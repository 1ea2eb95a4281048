"""In-process A/B of encode kernel paths on the same buffers: 1M packets at (10,3,3) by default,
alternating batches, median per path.
  python tools/enc_paths_ab.py [--paths generic,tile] [--tbn 10,3,3] [--packets 1000010] [--env VAR=a|b]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--paths", default="generic,tile")
ap.add_argument("--tbn", default="10,3,3")
ap.add_argument("--packets", type=int, default=1_000_010)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--reps", type=int, default=7)
ap.add_argument("--env", default="", help="VAR=v1|v2|...: extra variants of the last path")
ap.add_argument("--nocheck", action="store_true", help="timing experiments whose outputs differ")
args = ap.parse_args()
T, B, N = map(int, args.tbn.split(","))
torch.cuda.set_device(0)
P = args.packets
payload = fill_payload(0, P, 300, 0x5EED)
variants = [(p, None) for p in args.paths.split(",")]
if args.env:
    var, vals = args.env.split("=")
    last = variants.pop()[0]
    variants += [(last, (var, v)) for v in vals.split("|")]
codecs = {}
outs = {}
for path, env in variants:
    c = Codec(300, T, B, N)
    c.set_encode_path(path)
    codecs[(path, env)] = c
cw = torch.empty((P, codecs[variants[0]].CW), dtype=torch.uint8, device="cuda")
wl = torch.empty(P, dtype=torch.int32, device="cuda")
ref = None
for v in variants:
    if v[1]:
        os.environ[v[1][0]] = v[1][1]
    cw.zero_()
    codecs[v].encode(payload, out=cw, out_len=wl)
    torch.cuda.synchronize()
    h = (cw.clone(), wl.clone())
    if ref is None:
        ref = h
    elif not args.nocheck:
        assert torch.equal(ref[0], h[0]) and torch.equal(ref[1], h[1]), f"{v} differs from {variants[0]}"
print("outputs identical across", [f"{p}{'' if e is None else ':' + '='.join(e)}" for p, e in variants], flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = {v: [] for v in variants}
for _ in range(args.reps):
    for v in variants:
        if v[1]:
            os.environ[v[1][0]] = v[1][1]
        c = codecs[v]
        c.encode(payload, out=cw, out_len=wl)
        e0.record()
        for _ in range(args.iters):
            c.encode(payload, out=cw, out_len=wl)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) * 1e3 / args.iters)
alg = (300 + codecs[variants[0]].CW) * P
for v, x in res.items():
    us = sorted(x)[len(x) // 2]
    name = v[0] + ("" if v[1] is None else ":" + "=".join(v[1]))
    print(f"{name:24s} {us:8.1f} us  {alg / us / 1e3:7.1f} GB/s algorithmic  (min {min(x):.1f})", flush=True)
