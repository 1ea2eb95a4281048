"""Type-2 relay chain alone (tiled kernels), 360 000 packets of (10,3,3) with bin/erasure.bin on hop 1
and bin/erasure2.bin on hop 2: for rocprofv3 passes (kernel trace, PMC).   python tools/swdf_bench.py [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.relay import SymbolWiseRelay  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
P, L = 360000, 300
torch.cuda.set_device(0)
c = Codec(L, 10, 3, 3)
cw, _ = c.encode(fill_payload(0, P, L, 0x5EED))
e1 = torch.from_numpy(load_pattern("bin_erasure")[:P].astype(np.uint8).copy()).cuda()
e2 = torch.from_numpy(load_pattern("bin_erasure2")[:P].astype(np.uint8).copy()).cuda()
r2 = SymbolWiseRelay(L, 10, 3, 10, 3)
frames, fl = r2.relay(cw, e1)
out, dfl = r2.destination(frames, e2)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    r2.relay(cw, e1, frames, fl)
    r2.destination(frames, e2, out, dfl)
torch.cuda.synchronize()
print(f"type 2 relay + destination: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms per 360000 packets")
