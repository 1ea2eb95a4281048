"""Decode copy kernel: tile size A/B (FEC_COPY_TILE = packets per workgroup) in one process on the
same buffers, alone and right after the encoder (as in the bench step)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import L, stream_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

torch.cuda.set_device(0)
TBN = tuple(int(x) for x in os.environ.get("TBN", "10,3,3").split(","))
P, T = int(os.environ.get("PACKETS", "1000000")), TBN[0]
Pf = P + T
tiles = [int(x) for x in (sys.argv[1:] or ["64", "32", "16"])]
codecs = {}
for tp in tiles:
    os.environ["FEC_COPY_TILE"] = str(tp)
    codecs[tp] = Codec(L, *TBN)
payload = fill_payload(0, Pf, L, 0x5EED)
er = torch.from_numpy(stream_pattern(Pf, 0)).cuda()
c0 = codecs[tiles[0]]
cw, wl = c0.encode(payload)
ref_out, ref_len = c0.copy(cw, er)
out = torch.empty((P, L), dtype=torch.uint8, device="cuda")
ol = torch.empty(P, dtype=torch.int32, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for tp, c in codecs.items():
    c.copy(cw, er, out=out, out_len=ol)
    torch.cuda.synchronize()
    assert torch.equal(out, ref_out) and torch.equal(ol, ref_len), tp

res = {}
for rnd in range(5):
    for tp, c in codecs.items():
        for mode in ["alone", "after_encode"]:
            t = []
            for _ in range(10):
                if mode == "after_encode":
                    c.encode(payload, out=cw, out_len=wl)
                e0.record()
                c.copy(cw, er, out=out, out_len=ol)
                e1.record()
                torch.cuda.synchronize()
                t.append(e0.elapsed_time(e1) * 1e3)
            res.setdefault((tp, mode), []).append(sorted(t)[5])
for (tp, mode), v in res.items():
    print(f"{TBN} tile {tp:3d} {mode:13s}: median {sorted(v)[2]:.1f} us  (rounds {', '.join(f'{x:.1f}' for x in v)})")
