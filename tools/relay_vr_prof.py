"""The batched adaptive relay (fec_relay_vr, AdaptiveRelay) on config 4's schedule, 360 000 seqs, hops
bin/erasure.bin / bin/erasure2.bin: wall time per run of each type, for a rocprofv3 kernel trace.
    python tools/relay_vr_prof.py [reps] [types]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import fill_payload  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.relay import AdaptiveRelay, relay_digest  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
types = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [2, 3]
g = json.load(open(os.path.join(ROOT, "tests", "golden", "relay_vr_360k.json")))
P = g["P"]
torch.cuda.set_device(0)
payload = fill_payload(0, P, 300, 0x5EED)
e1, e2 = load_pattern("bin_erasure")[:P], load_pattern("bin_erasure2")[:P]
for t in types:
    r = AdaptiveRelay(t, 300, g["schedule"], P)
    frames, flen, out, flags = r.run(payload, e1, e2)
    torch.cuda.synchronize()
    ok = [f"{c:08x}" for c in relay_digest(frames, flen, out, flags)] == g[f"type{t}"]["blocks"]
    t0 = time.perf_counter()
    for _ in range(reps):
        r.run(payload, e1, e2)
    torch.cuda.synchronize()
    print(f"type {t}: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms per run, verified {ok}", flush=True)
