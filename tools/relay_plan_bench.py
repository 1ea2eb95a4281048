"""Host planners of the state-dependent relay (type 3) alone, on the CPU: relay and destination
plans of 360 000 packets ((10,3) -> (10,3), hop 1 bin/erasure.bin, hop 2 bin/erasure2.bin), time per
plan and a digest of the plans (to compare builds).   python tools/relay_plan_bench.py [reps]"""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fec_erasure_code_unit_test_relay_amd.relay import StateDependentRelay  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
P = 360000
e1 = load_pattern("bin_erasure")[:P].astype(np.uint8)
e2 = load_pattern("bin_erasure2")[:P].astype(np.uint8)
r = StateDependentRelay(300, 10, 3, 10, 3)
ids, rec = r.relay_plan(e1)
hdr = rec[ids, :11]
dids, drec, dfl = r.dest_plan(e2, hdr)
h = hashlib.sha256()
for a in (ids, rec, dids, drec, dfl):
    h.update(np.ascontiguousarray(a).tobytes())
best_r = best_d = 1e9
for _ in range(reps):
    t0 = time.perf_counter()
    r.relay_plan(e1)
    t1 = time.perf_counter()
    r.dest_plan(e2, hdr)
    t2 = time.perf_counter()
    best_r, best_d = min(best_r, (t1 - t0) / 2), min(best_d, (t2 - t1) / 2)  # each wrapper plans twice
print(f"relay plan {best_r * 1e3:.1f} ms, destination plan {best_d * 1e3:.1f} ms per {P} packets; "
      f"records {len(rec)} / {len(drec)}; digest {h.hexdigest()[:16]}")
