"""In-process A/B of the bench step (encode + fec_decode_batch) over codec switches:
  python tools/step_ab.py dedup=1 dedup=0 plan=fast plan=generic copy=fast copy=generic
  combo=copy:fast,env:FEC_COPY_WPC:8   (settings persist: give every variant all its switches)"""
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


def apply(cfg):
    k, v = cfg.split("=")
    if k == "dedup":
        c.set_episode_dedup(v == "1")
    elif k == "plan":
        c.set_plan_path(v)
    elif k == "copy":
        c.set_copy_path(v)
    elif k == "combo":  # combo=copy:fast,env:FEC_COPY_WPC:16
        for part in v.split(","):
            kk, vv = part.split(":", 1)
            apply(f"{kk}={vv}")
    elif k == "env":
        var, val = v.split(":")
        os.environ[var] = val


def step():
    c.encode(payload, out=cw, out_len=wl)
    c.decode(cw, er, out=out, out_len=ol)


res = {cfg: [] for cfg in sys.argv[1:]}
for rnd in range(5):
    for cfg in res:
        apply(cfg)
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        res[cfg].append((time.perf_counter() - t0) / 20 * 1e3)
        ok = ol != 0
        assert torch.equal(out[ok], payload[:P][ok]) and int((~ok).sum()) == 11851
print("  ".join(f"{k}: {sorted(v)[2]:.4f} ms ({P * L / sorted(v)[2] / 1e-3 / 2**30:.1f} GiB/s)" for k, v in res.items()))
