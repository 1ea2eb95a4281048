"""Relay chains (RELAYING_TYPE 2 and 3), 360 000 packets of (10,3,3) with bin/erasure.bin on hop 1 and
bin/erasure2.bin on hop 2: time of each batched call, and of type 3's host planners alone.
    python tools/relay_prof.py [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.relay import StateDependentRelay, SymbolWiseRelay  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
P, L = 360000, 300
torch.cuda.set_device(0)
c = Codec(L, 10, 3, 3)
cw, _ = c.encode(fill_payload(0, P, L, 0x5EED))
e1 = load_pattern("bin_erasure")[:P].astype(np.uint8)
e2 = load_pattern("bin_erasure2")[:P].astype(np.uint8)


def t(name, fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = fn()
    torch.cuda.synchronize()
    print(f"{name:34s} {(time.perf_counter() - t0) / reps * 1e3:9.3f} ms", flush=True)
    return r


r2 = SymbolWiseRelay(L, 10, 3, 10, 3)
e1d, e2d = torch.from_numpy(e1.copy()).cuda(), torch.from_numpy(e2.copy()).cuda()
f2, _ = t("type 2 relay", lambda: r2.relay(cw, e1d))
t("type 2 destination", lambda: r2.destination(f2, e2d))
r3 = StateDependentRelay(L, 10, 3, 10, 3)
f3 = t("type 3 relay (planner + kernel)", lambda: r3.relay(cw, e1))
t("type 3 destination (planner + kernel)", lambda: r3.destination(f3, e2))
t("type 3 relay planner alone", lambda: r3.relay_plan(e1))
hdr = f3[:, 2:13].cpu().numpy().copy()
t("type 3 destination planner alone", lambda: r3.dest_plan(e2, hdr))
