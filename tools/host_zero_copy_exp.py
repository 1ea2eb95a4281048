"""Host-inclusive leg with the kernels reading and writing pinned host memory directly (no SDMA
copies): encode from the host payload rows into host codeword rows, decode from the host codeword
rows (erasure flags up once, on the device) into host payload rows; both PCIe directions are in
flight inside each kernel.  Compared with bench.py's SDMA pipeline on the same buffers; the outputs
are checked against the device-resident decode.
  python tools/host_zero_copy_exp.py [--packets 1000000] [--reps 3]"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import L, stream_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402
from fec_erasure_code_unit_test_relay_amd._lib import lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--packets", type=int, default=1_000_000)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--no-pipe", action="store_true")
args = ap.parse_args()
torch.cuda.set_device(0)
T = 10
P = args.packets
Pf = P + T
c = Codec(L, 10, 3, 3)
vp = ctypes.c_void_p
payload = fill_payload(0, Pf, L, 0x5EED)
er = torch.from_numpy(stream_pattern(Pf, 0)).cuda()
# device-resident reference
cw_d = torch.empty((Pf, c.CW), dtype=torch.uint8, device="cuda")
wl_d = torch.empty(Pf, dtype=torch.int32, device="cuda")
out_d = torch.empty((P, L), dtype=torch.uint8, device="cuda")
ol_d = torch.empty(P, dtype=torch.int32, device="cuda")
c.encode(payload, out=cw_d, out_len=wl_d)
c.decode(cw_d, er, out=out_d, out_len=ol_d)
torch.cuda.synchronize()
# pinned host buffers (the socket side), device-mapped under unified addressing
h_payload = payload.cpu().pin_memory()
h_cw = torch.empty((Pf, c.CW), dtype=torch.uint8).pin_memory()
h_wl = torch.empty(Pf, dtype=torch.int32).pin_memory()
h_out = torch.empty((P, L), dtype=torch.uint8).pin_memory()
h_ol = torch.empty(P, dtype=torch.int32).pin_memory()
ws = c.workspace(Pf)
st = vp(torch.cuda.current_stream().cuda_stream)


def p(t):
    return vp(t.data_ptr())


def zero_copy_step():
    assert lib().fec_encode_batch(c._h, p(h_payload), None, 0, Pf, p(h_cw), p(h_wl), st) == 0
    assert lib().fec_decode_batch(c._h, p(h_cw), p(er), Pf, p(h_out), p(h_ol), p(ws), ws.numel(), st) == 0


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


dt = timed(zero_copy_step, args.reps)
ok = bool(torch.equal(h_out, out_d.cpu())) and bool(torch.equal(h_ol, ol_d.cpu())) and bool(
    torch.equal(h_cw, cw_d.cpu()))
print(f"zero-copy host->host encode+decode: {dt * 1e3:.3f} ms, {P * L / dt / 2**30:.2f} GiB/s, "
      f"outputs {'equal' if ok else 'DIFFER'} to the device-resident run", flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, fn in (("encode", lambda: lib().fec_encode_batch(c._h, p(h_payload), None, 0, Pf, p(h_cw), p(h_wl), st)),
                 ("decode", lambda: lib().fec_decode_batch(c._h, p(h_cw), p(er), Pf, p(h_out), p(h_ol), p(ws),
                                                           ws.numel(), st))):
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(args.reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"  {name} alone: {e0.elapsed_time(e1) / args.reps:.3f} ms", flush=True)

# Pipelined: encode chunk i+1 (PCIe mostly device->host) on one stream while chunk i is decoded
# (mostly host->device) on another by the continuing decoder -- the two directions balance.
from fec_erasure_code_unit_test_relay_amd import DecodeStream  # noqa: E402
import numpy as np  # noqa: E402

pat = er.cpu().numpy()
h_er = er.cpu().pin_memory()
s_a, s_b = torch.cuda.Stream(), torch.cuda.Stream()
CW = c.CW


def zero_copy_pipelined(NC):
    cuts = [Pf * i // NC for i in range(NC + 1)]
    ds = DecodeStream(c)
    cur = torch.cuda.current_stream()
    s_a.wait_stream(cur)
    s_b.wait_stream(cur)
    sa, sb = vp(s_a.cuda_stream), vp(s_b.cuda_stream)
    n0 = 0
    for i in range(NC):
        a, b = cuts[i], cuts[i + 1]
        h = min(a, c.n - 1)
        with torch.cuda.stream(s_a):
            assert lib().fec_encode_batch(c._h, vp(h_payload.data_ptr() + a * L), None, h, b - a,
                                          vp(h_cw.data_ptr() + a * CW), vp(h_wl.data_ptr() + 4 * a), sa) == 0
            ev = torch.cuda.Event()
            ev.record()
        with torch.cuda.stream(s_b):
            s_b.wait_event(ev)
            n = ctypes.c_int64()
            assert lib().fec_decode_stream_push(
                c._h, ds._h, vp(h_cw.data_ptr() + a * CW), vp(h_er.data_ptr() + a), vp(pat.ctypes.data + a),
                b - a, a, vp(h_out.data_ptr() + n0 * L), vp(h_ol.data_ptr() + 4 * n0), ctypes.byref(n),
                p(ws), ws.numel(), sb) == 0
            n0 += n.value
    cur.wait_stream(s_a)
    cur.wait_stream(s_b)
    return n0


for NC in (() if args.no_pipe else (2, 4, 8, 16)):
    h_out.zero_()
    h_ol.zero_()
    dt = timed(lambda: zero_copy_pipelined(NC), args.reps)
    ok = bool(torch.equal(h_out, out_d.cpu())) and bool(torch.equal(h_ol, ol_d.cpu()))
    print(f"zero-copy pipelined NC={NC}: {dt * 1e3:.3f} ms, {P * L / dt / 2**30:.2f} GiB/s, "
          f"outputs {'equal' if ok else 'DIFFER'}", flush=True)
