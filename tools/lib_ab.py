"""In-process A/B of two builds of the library (e.g. libfec_amd.so vs libfec_amd_b.so built with
EXTRA=-D...): encode of 1M packets at (10,3,3), alternating batches, median per build.
  python tools/lib_ab.py fec_erasure_code_unit_test_relay_amd/libfec_amd.so fec_erasure_code_unit_test_relay_amd/libfec_amd_b.so"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402  (load torch's HIP runtime first)

torch.cuda.set_device(0)
from fec_erasure_code_unit_test_relay_amd import fill_payload  # noqa: E402

libs = [ctypes.CDLL(os.path.abspath(p)) for p in sys.argv[1:]]
vp = ctypes.c_void_p
P = 1_000_010
payload = fill_payload(0, P, 300, 0x5EED)
codecs = []
for L in libs:
    L.fec_codec_create.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(vp)]
    L.fec_encode_batch.argtypes = [vp, vp, vp, ctypes.c_int64, ctypes.c_int64, vp, vp, vp]
    h = vp()
    assert L.fec_codec_create(300, 10, 3, 3, ctypes.byref(h)) == 0
    codecs.append(h)
# one output buffer for every build: timings depend on where the buffers land in HBM
cw = torch.empty((P, 418), dtype=torch.uint8, device="cuda")
wl = torch.empty(P, dtype=torch.int32, device="cuda")
cws = [cw for _ in libs]
wls = [wl for _ in libs]
st = vp(torch.cuda.current_stream().cuda_stream)


def enc(i):
    assert libs[i].fec_encode_batch(codecs[i], vp(payload.data_ptr()), None, 0, P, vp(cws[i].data_ptr()),
                                    vp(wls[i].data_ptr()), st) == 0


e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = [[] for _ in libs]
for rnd in range(9):
    for i in range(len(libs)):
        enc(i)
        e0.record()
        for _ in range(20):
            enc(i)
        e1.record()
        torch.cuda.synchronize()
        res[i].append(e0.elapsed_time(e1) * 1e3 / 20)
torch.cuda.synchronize()
outs = []
for i in range(len(libs)):
    cw.zero_()
    enc(i)
    torch.cuda.synchronize()
    outs.append((cw.clone(), wl.clone()))
same = all(torch.equal(outs[0][0], c) and torch.equal(outs[0][1], w) for c, w in outs[1:])
print("  ".join(f"{os.path.basename(p)}: {sorted(r)[4]:.1f} us" for p, r in zip(sys.argv[1:], res)), "identical" if same else "DIFFER")
