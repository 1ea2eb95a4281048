"""Graph-replayed parts of the bench step (no host launch gaps), one process, same buffers:
  encode | plan | copy | plan beside copy | recover | decode | step, each captured once and
  replayed; environment switches (FEC_*) are read at capture time.
  python tools/graph_parts.py [--packets 1000000] [--tbn 10,3,3] [--env FEC_PLAN_GRID=1024 ...]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import L, stream_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--packets", type=int, default=1_000_000)
ap.add_argument("--tbn", default="10,3,3")
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--env", nargs="*", default=[], help="VAR=VALUE settings, one variant each ('-' = none)")
args = ap.parse_args()
T, B, N = map(int, args.tbn.split(","))
torch.cuda.set_device(0)
P = args.packets
Pf = P + T
c = Codec(L, T, B, N)
payload = fill_payload(0, Pf, L, 0x5EED)
er = torch.from_numpy(stream_pattern(Pf, 0)).cuda()
cw = torch.empty((Pf, c.CW), dtype=torch.uint8, device="cuda")
wl = torch.empty(Pf, dtype=torch.int32, device="cuda")
out = torch.empty((P, L), dtype=torch.uint8, device="cuda")
ol = torch.empty(P, dtype=torch.int32, device="cuda")
c.workspace(Pf)
side = torch.cuda.Stream()
c.encode(payload, out=cw, out_len=wl)
torch.cuda.synchronize()


def plan_beside_copy():
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        c.plan(er)
    c.copy(cw, er, out=out, out_len=ol)
    cur.wait_stream(side)


PARTS = [("encode", lambda: c.encode(payload, out=cw, out_len=wl)), ("plan", lambda: c.plan(er)),
         ("copy", lambda: c.copy(cw, er, out=out, out_len=ol)), ("plan||copy", plan_beside_copy),
         ("recover", lambda: c.recover(cw, out, ol)), ("decode", lambda: c.decode(cw, er, out=out, out_len=ol)),
         ("step", lambda: (c.encode(payload, out=cw, out_len=wl), c.decode(cw, er, out=out, out_len=ol)))]


def capture(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()  # warm-up outside the capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def timed(g, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    return sorted(ts)[2]


for variant in (args.env or ["-"]):
    saved = dict(os.environ)
    if variant != "-":
        for kv in variant.split(","):
            k, v = kv.split("=", 1)
            os.environ[k] = v
    c.set_copy_path(os.environ.get("FEC_GP_COPY", "auto"))  # e.g. FEC_GP_COPY=generic
    graphs = [(name, capture(fn)) for name, fn in PARTS]
    res = {name: timed(g, args.reps) for name, g in graphs}
    c.decode(cw, er, out=out, out_len=ol)
    torch.cuda.synchronize()
    ok = ol != 0
    assert torch.equal(out[ok], payload[:P][ok])
    print(f"[{variant}] P={P} tbn={args.tbn} " + "  ".join(f"{k}: {v:.1f}" for k, v in res.items()) + " us",
          flush=True)
    os.environ.clear()
    os.environ.update(saved)
