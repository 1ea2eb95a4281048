"""Continuing decode vs one-shot decode: where do rows differ (relative to the push cuts)?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import fec_erasure_code_unit_test_relay_amd as fec  # noqa: E402
from conftest import load_pattern  # noqa: E402

torch.cuda.set_device(0)
L, T, B, N = 300, 10, 3, 3
P = 12000
pat = load_pattern("erasure50")[:P + T].astype(np.uint8)
c = fec.Codec(L, T, B, N)
payload = fec.fill_payload(0, P + T, L, 0x5EED)
cw, _ = c.encode(payload)
er = torch.from_numpy(pat).cuda()
ref, ref_len = c.decode(cw, er)
rl = ref_len.cpu().numpy()
for cuts in ([0, 5000, P + T], [0, 3000, 7000, P + T], [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 100, P + T]):
    ds = fec.DecodeStream(c)
    outs, lens = [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        o, ln = ds.push(cw[0:b], er[0:b], pat[0:b], history=a)
        torch.cuda.synchronize()
        cons, lc = ds.state()
        print(f"push [{a},{b}): {o.shape[0]} rows, restart at {lc}")
        outs.append(o.clone())
        lens.append(ln.clone())
    out = torch.cat(outs)
    ln = torch.cat(lens).cpu().numpy()
    bad = np.flatnonzero(ln != rl)
    badd = np.flatnonzero((out != ref).any(dim=1).cpu().numpy())
    print("cuts", cuts[:6], "len mismatches:", len(bad), bad[:10].tolist(), "got", ln[bad[:10]].tolist(),
          "want", rl[bad[:10]].tolist(), "erased?", pat[bad[:10]].tolist())
    print("   data mismatches:", len(badd), badd[:10].tolist())
