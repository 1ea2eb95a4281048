"""Diagnose the decode: episode list, recovered set and bytes vs host planner / oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from conftest import load_pattern  # noqa: E402
import fec_erasure_code_unit_test_relay_amd as fec  # noqa: E402

torch.cuda.set_device(0)
L = 300
for (T, B, N), P in [((10, 5, 2), 8000), ((10, 3, 3), 8000)]:
    pat = load_pattern("bin_erasure")[:P + T].copy()
    e = pat.astype(bool)
    res = sorted(t for t in range(P + T) if e[t] and not e[max(0, t - T - 1):t].any())
    c = fec.Codec(L, T, B, N)
    er = torch.from_numpy(pat).cuda()
    c.plan(er)
    torch.cuda.synchronize()
    ws = c._ws.cpu().numpy()
    cnt = ws[:64].view(np.int32)
    got = sorted(ws[256:256 + 4 * int(cnt[0])].view(np.int32).tolist())
    print((T, B, N), "episodes", int(cnt[0]), "expected", len(res), "list equal", got == res, flush=True)
    if got != res:
        print("  missing", sorted(set(res) - set(got))[:20], "extra", sorted(set(got) - set(res))[:20])
        print("  STOP: episode list wrong, not running the decode")
        break
    payload = fec.fill_payload(0, P + T, L, 0x5EED)
    cw, _ = c.encode(payload)
    out, ln = c.decode(cw, er)
    torch.cuda.synchronize()
    eps, rec, lost = c.counters()
    fate = fec.plan_host(L, T, B, N, pat)
    lnh = ln.cpu().numpy()
    ref = oracle.run_stream(L, T, B, N, P, pat, want_data=True)
    print("  recovered gpu", rec, "host", int((fate == 2).sum()), "lost gpu", lost, "host",
          int((fate == 3).sum()), flush=True)
    bad = np.flatnonzero(lnh != ref["out_len"])
    print("  len mismatches", bad.size, bad[:20])
    bytes_bad = np.flatnonzero((out.cpu().numpy() != ref["out_data"]).any(axis=1))
    print("  rows with byte mismatch", bytes_bad.size, bytes_bad[:10], flush=True)
