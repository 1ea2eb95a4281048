"""Config 4 encode through the tile path vs the generic kernel (FEC_VR_NO_TILE): compare the
codeword arrays row by row and report mismatches by instance tuple.  python tools/debug_vr_tile.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import fill_payload  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.vr import VrPlan  # noqa: E402

torch.cuda.set_device(0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
pat = load_pattern("bin_erasure")
P = 360000
os.environ.pop("FEC_VR_NO_TILE", None)
v_tile = VrPlan(pat, P)
os.environ["FEC_VR_NO_TILE"] = "1"
v_gen = VrPlan(pat, P)
os.environ.pop("FEC_VR_NO_TILE", None)
payload = fill_payload(0, v_tile.sent, 300, 0x5EED)
ref = v_gen.encode(payload)
torch.cuda.synchronize()
enc = v_tile.encoders
fr = v_tile.frames
for r in range(reps):
    got = v_tile.encode(payload)
    torch.cuda.synchronize()
    for name, a, b in (("cur", got[0], ref[0]), ("len_cur", got[1], ref[1]), ("old", got[2], ref[2]),
                       ("len_old", got[3], ref[3])):
        if a.dim() == 2:
            bad = (a != b).any(dim=1).cpu().numpy()
        else:
            bad = (a != b).cpu().numpy()
        idx = np.flatnonzero(bad)
        if idx.size:
            col = 4 if name in ("cur", "len_cur") else 5
            tup = {}
            for s in idx[:2000]:
                e = fr[s, col]
                t = tuple(int(x) for x in enc[e, :3]) if e >= 0 else None
                tup[t] = tup.get(t, 0) + 1
            print(f"rep {r}: {name}: {idx.size} rows differ, first {idx[:8].tolist()}, by tuple {tup}", flush=True)
            if a.dim() == 2:
                s = int(idx[0])
                d = np.flatnonzero((a[s] != b[s]).cpu().numpy())
                print(f"   row {s}: bytes differ at {d[:16].tolist()} (of {d.size}); frame {fr[s].tolist()}", flush=True)
        else:
            print(f"rep {r}: {name}: identical", flush=True)
