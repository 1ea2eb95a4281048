"""In-process A/B of the tile encoder specialised on L = 300 against the runtime-L instance (same
buffers, alternating graph-replayed batches): python tools/enc_ab_L.py [--tbn 10,3,3]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tbn", default="10,3,3")
ap.add_argument("--packets", type=int, default=1_000_010)
args = ap.parse_args()
T, B, N = map(int, args.tbn.split(","))
torch.cuda.set_device(0)
L = 300
codecs = {}
os.environ["FEC_TILE_RUNTIME_L"] = "1"
codecs["runtime L"] = Codec(L, T, B, N)
os.environ.pop("FEC_TILE_RUNTIME_L")
codecs["L = 300"] = Codec(L, T, B, N)
for name, c in codecs.items():
    print(name, c.info()["encode_kernel"], flush=True)
P = args.packets
payload = fill_payload(0, P, L, 0x5EED)
c0 = next(iter(codecs.values()))
cw = torch.empty((P, c0.CW), dtype=torch.uint8, device="cuda")
wl = torch.empty(P, dtype=torch.int32, device="cuda")
ref = None
graphs = {}
for name, c in codecs.items():
    c.encode(payload, out=cw, out_len=wl)
    torch.cuda.synchronize()
    if ref is None:
        ref = (cw.clone(), wl.clone())
    else:
        assert torch.equal(cw, ref[0]) and torch.equal(wl, ref[1]), name
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        c.encode(payload, out=cw, out_len=wl)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        c.encode(payload, out=cw, out_len=wl)
    graphs[name] = g
res = {k: [] for k in graphs}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rnd in range(7):
    for name, g in graphs.items():
        g.replay()
        e0.record()
        for _ in range(20):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name].append(e0.elapsed_time(e1) * 1e3 / 20)
print("  ".join(f"{k}: {sorted(v)[3]:.1f} us" for k, v in res.items()), flush=True)
