"""Bench step (encode + fec_decode_batch, eager launches) under environment settings read at each
launch (FEC_TILE_NT, FEC_COPY_NT, ...), one process, same buffers; every variant's
outputs are checked (round trip + lost count).  Per-kernel event times are printed beside the step.
  python tools/step_env_ab.py "" "FEC_TILE_NT=2" "FEC_COPY_NT=1,FEC_TILE_NT=2" """
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
settings = sys.argv[1:] or [""]
keys = {kv.split("=")[0] for s in settings for kv in s.split(",") if kv}


def apply(sset):
    for k in keys:
        os.environ.pop(k, None)
    for kv in sset.split(","):
        if kv:
            k, v = kv.split("=")
            os.environ[k] = v


def step():
    c.encode(payload, out=cw, out_len=wl)
    c.decode(cw, er, out=out, out_len=ol)


t_end = time.perf_counter() + 1.0
while time.perf_counter() < t_end:
    step()
    torch.cuda.synchronize()
res = {s: [] for s in settings}
kern = {s: {} for s in settings}
for rnd in range(6):
    for sset in settings:
        apply(sset)
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        res[sset].append((time.perf_counter() - t0) / 20 * 1e3)
        ok = ol != 0
        assert torch.equal(out[ok], payload[:P][ok]) and int((~ok).sum()) == 11851, sset
        c.timing(True)
        for _ in range(10):
            step()
        for k, (ms, n) in c.collect_timing().items():
            if n:
                kern[sset].setdefault(k, []).append(ms / n * 1e3)
        c.timing(False)
for sset, v in res.items():
    m = sorted(v)[len(v) // 2]
    ks = "  ".join(f"{k.replace('fec_', '').replace('_kernel', '')} {sorted(x)[len(x) // 2]:.1f}" for k, x in kern[sset].items())
    print(f"[{sset or 'default'}] {m:.4f} ms/step ({P * L / m / 1e-3 / 2**30:.1f} GiB/s); us: {ks}", flush=True)
