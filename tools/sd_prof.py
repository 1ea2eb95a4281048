"""Type-3 relay chain kernels alone (for rocprofv3 --kernel-trace --stats): (10,3,3) codewords of
360 000 packets -> relay -> destination, hop erasures bin/erasure.bin / bin/erasure2.bin, N times.
    python tools/sd_prof.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.relay import StateDependentRelay  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
torch.cuda.set_device(0)
P, L = 360000, 300
c = Codec(L, 10, 3, 3)
payload = fill_payload(0, P, L, 0x5EED)
cw, _ = c.encode(payload)
e1 = load_pattern("bin_erasure")[:P].astype(np.uint8)
e2 = load_pattern("bin_erasure2")[:P].astype(np.uint8)
r = StateDependentRelay(L, 10, 3, 10, 3)
frames = r.relay(cw, e1)
out, fl = r.destination(frames, e2)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    frames = r.relay(cw, e1)
    out, fl = r.destination(frames, e2)
torch.cuda.synchronize()
print(f"type 3 chain: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms", flush=True)
