"""Probe of the one-stream tile encoder at the adaptive relay's batch shapes: (T,N) = (10,0), (10,1),
(10,5) over 212 000 / 108 000 / 106 000 rows alone on the GPU (the relay runs them side by side),
all rows at length L, or with the relay's zero-length gap rows (33 in front of every ~230 rows), and
(10,3) at L = 300 (the specialised kernel) for scale.  CUDA-event time per encode, median of 20.
    python tools/enc_rl_probe.py"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

torch.cuda.set_device(0)
L = 300
for (T, N, R) in [(10, 3, 212000), (10, 0, 212000), (10, 1, 108000), (10, 5, 106000)]:
    c = Codec(L, T, N, N)
    pay = fill_payload(0, R, L, 0x5EED)
    full = torch.full((R,), L, dtype=torch.int32, device="cuda")
    gap = full.clone()
    idx = torch.arange(R, device="cuda")
    gap[(idx % 263) < 33] = 0
    out, ol = c.encode(pay)
    res = {}
    for name, ln in (("no lengths", None), ("all L", full), ("gap rows", gap)):
        ts = []
        for _ in range(23):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            c.encode(pay, ln, out=out, out_len=ol)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        res[name] = statistics.median(ts[3:])
    print(f"(T,N)=({T},{N}) k={c.k} rows {R}: " + "  ".join(f"{k}: {v:.1f} us" for k, v in res.items()), flush=True)
