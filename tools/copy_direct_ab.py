"""Copy kernel A/B (same process, same buffers): LDS output tile vs direct payload stores
(FEC_COPY_DIRECT), tile of 32 / 64 packets (FEC_COPY_TILE).  Times the copy alone (50 back-to-back
launches between two events) and the bench step (encode + decode), checks the outputs are equal."""
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
payload = fill_payload(0, Pf, L, 0x5EED)
er = torch.from_numpy(stream_pattern(Pf, 0)).cuda()
variants = [(int(v.split(":")[0]), int(v.split(":")[1])) for v in sys.argv[1:]] or [(32, 0), (32, 1), (64, 1), (16, 1), (32, 0), (32, 1)]
ref = None
for tp, d in variants:
    os.environ["FEC_COPY_TILE"] = str(tp)
    os.environ["FEC_COPY_DIRECT"] = str(d)
    c = Codec(L, 10, 3, 3)
    cw = torch.empty((Pf, c.CW), dtype=torch.uint8, device="cuda")
    wl = torch.empty(Pf, dtype=torch.int32, device="cuda")
    out = torch.empty((P, L), dtype=torch.uint8, device="cuda")
    ol = torch.empty(P, dtype=torch.int32, device="cuda")
    c.workspace(Pf)

    def step():
        c.encode(payload, out=cw, out_len=wl)
        c.decode(cw, er, out=out, out_len=ol)

    for _ in range(200):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        step()
    e1.record()
    torch.cuda.synchronize()
    st = e0.elapsed_time(e1) / 50
    if ref is None:
        ref = (out.clone(), ol.clone())
    same = torch.equal(out, ref[0]) and torch.equal(ol, ref[1])
    for _ in range(5):
        c.copy(cw, er, out=out, out_len=ol)
    e0.record()
    for _ in range(50):
        c.copy(cw, er, out=out, out_len=ol)
    e1.record()
    torch.cuda.synchronize()
    cp = e0.elapsed_time(e1) / 50
    print(f"TP={tp:3d} direct={d}: copy {cp * 1e3:7.1f} us back-to-back, step {st:.4f} ms "
          f"({P * L / st / 1e-3 / 2**30:.1f} GiB/s), outputs equal: {same}", flush=True)
    del c
