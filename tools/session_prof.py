"""The two-hop relay session's byte work under a profiler: one warm-up run and `reps` timed runs of
each relay type over bin/erasure.bin / bin/erasure2.bin (Q = 360 020).  Run as
    rocprofv3 --kernel-trace --stats -d DIR -o session -- python3 tools/session_prof.py [reps]"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import fill_payload  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.relay import RelaySession  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
Q = 360020
e1, e2 = load_pattern("bin_erasure"), load_pattern("bin_erasure2")
pay = fill_payload(0, Q, 300, 0x5EED)
for t in (2, 3):
    s = RelaySession(t, Q, e1, e2)
    bufs = s.run(pay)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        s.run(pay, *bufs)
    torch.cuda.synchronize()
    print(f"type {t}: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms per run, lost {int(bufs[3].item())}, "
          f"{s.stats['lineages']} lineages (longest {s.stats['longest_lineage']}), {s.stats['relay_calls']} relay calls",
          flush=True)
