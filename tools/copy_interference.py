"""How much the planner chain beside the copy costs the copy: per-kernel event times of the bench
step (encode + fec_decode_batch) against encode + copy alone (no plan, no recovery), one process.
  python tools/copy_interference.py"""
import os
import sys

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


def full():
    c.encode(payload, out=cw, out_len=wl)
    c.decode(cw, er, out=out, out_len=ol)


def copy_only():
    c.encode(payload, out=cw, out_len=wl)
    c.copy(cw, er, out=out, out_len=ol)


def plan_serial():
    c.encode(payload, out=cw, out_len=wl)
    c.plan(er)
    c.copy(cw, er, out=out, out_len=ol)
    c.recover(cw, out=out, out_len=ol)


for rnd in range(3):
    for name, fn in (("step", full), ("encode+copy", copy_only), ("plan serial", plan_serial)):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        c.timing(True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        kt = c.collect_timing()
        c.timing(False)
        per = {k: round(ms / n * 1e3, 1) for k, (ms, n) in kt.items() if n}
        print(f"{name}: {e0.elapsed_time(e1) / 50:.4f} ms per step (timing on); us per launch {per}", flush=True)
