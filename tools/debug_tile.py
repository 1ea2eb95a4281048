"""Tile encode kernel vs the per-tile kernel: first mismatching packets for a few shapes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

torch.cuda.set_device(0)
L = 300
tbn = tuple(int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "10,3,3").split(","))
for P, use_len, hist in [(2500, False, 0), (2500, True, 0), (300000, False, 0), (300000, True, 0),
                         (300000, False, 64), (100000, False, 0), (20000, False, 0)]:
    rng = np.random.default_rng(17)
    lens = torch.from_numpy(rng.integers(0, L + 1, size=P).astype(np.int32)).cuda() if use_len else None
    payload = fill_payload(0, P, L, 23)
    res = []
    for path in ("fast", "tile"):
        c = Codec(L, *tbn)
        c.set_encode_path(path)
        if hist:
            cw, wl = c.encode(payload[P // 2 - hist:], None if lens is None else lens[P // 2 - hist:], history=hist)
        else:
            cw, wl = c.encode(payload, lens)
        torch.cuda.synchronize()
        res.append((cw.cpu().numpy(), wl.cpu().numpy()))
    (a, al), (b, bl) = res
    bad = np.flatnonzero((a != b).any(axis=1))
    badl = np.flatnonzero(al != bl)
    print(f"P={P} len={use_len} hist={hist}: {len(bad)} packets differ, {len(badl)} sizes differ", flush=True)
    if len(bad):
        print("  first bad packets:", bad[:12].tolist(), " R-mod:", (bad[:12] % 24).tolist())
        t = bad[0]
        cols = np.flatnonzero(a[t] != b[t])
        print("  packet", t, "bad byte columns:", cols[:40].tolist())
    if len(badl):
        print("  first bad sizes:", badl[:8].tolist(), al[badl[:8]].tolist(), bl[badl[:8]].tolist())
