"""Decode copy kernel time under environment settings read at launch (FEC_COPY_NT, FEC_CHUNK_DBG,
...), in one process on the same buffers.  Bytes are not checked (debug settings change them).
  python tools/copy_env_ab.py chunk "FEC_CHUNK_DBG=0" "FEC_CHUNK_DBG=1" "FEC_COPY_NT=0" """
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import L, stream_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

torch.cuda.set_device(0)
path, settings = sys.argv[1], sys.argv[2:]
P, T = 1_000_000, 10
Pf = P + T
c = Codec(L, 10, 3, 3)
c.set_copy_path(path)
payload = fill_payload(0, Pf, L, 0x5EED)
er = torch.from_numpy(stream_pattern(Pf, 0)).cuda()
cw, wl = c.encode(payload)
out = torch.empty((P, L), dtype=torch.uint8, device="cuda")
ol = torch.empty(P, dtype=torch.int32, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
keys = {kv.split("=")[0] for kv in settings}
res = {s: [] for s in settings}
for rnd in range(5):
    for sset in settings:
        for k in keys:
            os.environ.pop(k, None)
        for kv in sset.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
        t = []
        for _ in range(10):
            e0.record()
            c.copy(cw, er, out=out, out_len=ol)
            e1.record()
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1) * 1e3)
        res[sset].append(sorted(t)[5])
for sset, v in res.items():
    print(f"{path} {sset:30s}: median {sorted(v)[2]:.1f} us (rounds {', '.join(f'{x:.1f}' for x in v)})", flush=True)
