"""Bench step orchestrations, same process, same buffers, outputs checked:
  serial   -- encode; decode (plan beside the copy, recovery after it): the product's order
  early    -- plan + compaction start with the encoder (side stream); the recovery runs beside the
              copy, which leaves erased rows to it (FEC_COPY_SKIP=1: copy skips erased rows, the
              compaction zeroes the lost ones)
  earlyser -- plan beside the encoder, copy writes every row, recovery after the copy
  python tools/step_overlap2.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import L, stream_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

torch.cuda.set_device(0)
P, T = 1_000_000, 10
Pf = P + T
c = Codec(L, 10, 3, 3)
payload = fill_payload(0, Pf, L, 0x5EED)
er = torch.from_numpy(stream_pattern(Pf, 0)).cuda()
cw = torch.empty((Pf, c.CW), dtype=torch.uint8, device="cuda")
wl = torch.empty(Pf, dtype=torch.int32, device="cuda")
out = torch.empty((P, L), dtype=torch.uint8, device="cuda")
ol = torch.empty(P, dtype=torch.int32, device="cuda")
c.workspace(Pf)
side = torch.cuda.Stream()


def serial():
    os.environ.pop("FEC_COPY_SKIP", None)
    c.encode(payload, out=cw, out_len=wl)
    c.decode(cw, er, out=out, out_len=ol)


def early():
    os.environ["FEC_COPY_SKIP"] = "1"
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        c.plan(er, Pf)
    c.encode(payload, out=cw, out_len=wl)
    ev = torch.cuda.Event()
    ev.record()
    with torch.cuda.stream(side):
        side.wait_event(ev)
        c.recover(cw, out, ol)
    c.copy(cw, er, out=out, out_len=ol)
    cur.wait_stream(side)


def earlyser():
    os.environ.pop("FEC_COPY_SKIP", None)
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        c.plan(er, Pf)
    c.encode(payload, out=cw, out_len=wl)
    c.copy(cw, er, out=out, out_len=ol)
    cur.wait_stream(side)
    c.recover(cw, out, ol)


variants = {"serial": serial, "early": early, "earlyser": earlyser}
serial()
torch.cuda.synchronize()
ref_out, ref_ol = out.clone(), ol.clone()
for k, f in variants.items():
    out.fill_(0xCD)
    ol.fill_(-3)
    f()
    torch.cuda.synchronize()
    assert torch.equal(out, ref_out) and torch.equal(ol, ref_ol), k
t_end = time.perf_counter() + 1.0
while time.perf_counter() < t_end:
    serial()
    torch.cuda.synchronize()
res = {k: [] for k in variants}
for rnd in range(7):
    for k, f in variants.items():
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            f()
        torch.cuda.synchronize()
        res[k].append((time.perf_counter() - t0) / 20 * 1e3)
print("  ".join(f"{k}: {sorted(v)[3]:.4f} ms ({P * L / sorted(v)[3] / 1e-3 / 2**30:.1f} GiB/s)" for k, v in res.items()),
      flush=True)
