"""Per-packet latency of the reference-style streaming API (FEC_Encoder::onTransmit /
FEC_Decoder::onReceive over the C ABI, one GPU round trip per call), (10,3,3), 300-byte packets,
erasures from bin/erasure.bin."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import FEC_Decoder, FEC_Encoder  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402

torch.cuda.set_device(0)
P = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
pat = load_pattern("bin_erasure")[:P]
rng = np.random.default_rng(1)
data = rng.integers(0, 256, (P, 300), dtype=np.uint8)
enc, dec = FEC_Encoder(300, 10, 3, 3), FEC_Decoder(300, 10, 3, 3)
wire = []
t0 = time.perf_counter()
for s in range(P):
    wire.append(enc.onTransmit(data[s], 300, s))
t1 = time.perf_counter()
lost = 0
for s in range(P):
    cw, size = wire[s]
    out, p = dec.onReceive(None if pat[s] else cw, size, s, bool(pat[s]))
    if s >= 10:
        if p == 0:
            lost += 1
        else:
            assert (out[:300] == data[s - 10]).all()
t2 = time.perf_counter()
print(f"onTransmit {1e6 * (t1 - t0) / P:.1f} us/packet, onReceive {1e6 * (t2 - t1) / P:.1f} us/packet "
      f"({P} packets, {int(pat.sum())} erased, {lost} lost)")
