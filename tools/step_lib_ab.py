"""In-process A/B of the bench step (encode + fec_decode_batch, eager) between builds of the library,
same buffers, alternating batches of steps; median step time per build and the outputs compared.
  python tools/step_lib_ab.py fec_erasure_code_unit_test_relay_amd/libfec_amd.so fec_erasure_code_unit_test_relay_amd/libfec_amd_b.so"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402  (torch's HIP runtime first)

torch.cuda.set_device(0)
from bench import L, stream_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd import fill_payload  # noqa: E402

libs = [ctypes.CDLL(os.path.abspath(p)) for p in sys.argv[1:]]
vp, i64 = ctypes.c_void_p, ctypes.c_int64
P, T = 1_000_000, 10
Pf = P + T
payload = fill_payload(0, Pf, L, 0x5EED)
er = torch.from_numpy(stream_pattern(Pf, 0)).cuda()
cw = torch.empty((Pf, 418), dtype=torch.uint8, device="cuda")
wl = torch.empty(Pf, dtype=torch.int32, device="cuda")
out = torch.empty((P, L), dtype=torch.uint8, device="cuda")
ol = torch.empty(P, dtype=torch.int32, device="cuda")
codecs, wss = [], []
for lb in libs:
    lb.fec_codec_create.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(vp)]
    lb.fec_encode_batch.argtypes = [vp, vp, vp, i64, i64, vp, vp, vp]
    lb.fec_decode_batch.argtypes = [vp, vp, vp, i64, vp, vp, vp, i64, vp]
    lb.fec_decode_workspace_bytes.argtypes = [vp, i64]
    lb.fec_decode_workspace_bytes.restype = i64
    h = vp()
    assert lb.fec_codec_create(L, 10, 3, 3, ctypes.byref(h)) == 0
    codecs.append(h)
    wss.append(torch.empty(int(lb.fec_decode_workspace_bytes(h, Pf)), dtype=torch.uint8, device="cuda"))
st = vp(torch.cuda.current_stream().cuda_stream)


def step(i):
    lb, h, ws = libs[i], codecs[i], wss[i]
    assert lb.fec_encode_batch(h, vp(payload.data_ptr()), None, 0, Pf, vp(cw.data_ptr()), vp(wl.data_ptr()), st) == 0
    assert lb.fec_decode_batch(h, vp(cw.data_ptr()), vp(er.data_ptr()), Pf, vp(out.data_ptr()), vp(ol.data_ptr()),
                               vp(ws.data_ptr()), ws.numel(), st) == 0


outs = []
for i in range(len(libs)):
    for _ in range(300):
        step(i)
    torch.cuda.synchronize()
    outs.append((out.clone(), ol.clone()))
same = all(torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1]) for o in outs)
res = [[] for _ in libs]
for rnd in range(12):
    for i in range(len(libs)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(100):
            step(i)
        torch.cuda.synchronize()
        res[i].append((time.perf_counter() - t0) / 100 * 1e3)
for i, p in enumerate(sys.argv[1:]):
    r = sorted(res[i])
    print(f"{os.path.basename(p)}: step median {r[len(r) // 2]:.4f} ms, best {r[0]:.4f} ms", flush=True)
print("outputs equal" if same else "outputs DIFFER", flush=True)
