"""Config 4 device work only (for rocprofv3 --kernel-trace --stats): plan once, then encode +
decode of the schedule N times.   python tools/vr_prof.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import fill_payload  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.vr import VrPlan  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 5
if "--iters" in sys.argv:
    reps = int(sys.argv[sys.argv.index("--iters") + 1])
torch.cuda.set_device(0)
pat = load_pattern("bin_erasure")
P = 360000
v = VrPlan(pat, P)
pl = fill_payload(0, v.sent, 300, 0x5EED)
frames = v.alloc_frames(zero=False)
out = torch.empty((P, 300), dtype=torch.uint8, device="cuda")
ol = torch.empty(P, dtype=torch.int32, device="cuda")
for name, f in [("encode", lambda: v.encode(pl, frames=frames)),
                ("decode", lambda: v.decode(frames[0], frames[2], out=out, out_len=ol))]:
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"{name}: {(t1 - t0) / reps * 1e3:.3f} ms", flush=True)
    # host side alone: the calls enqueued behind a 20 ms spin kernel, so that none of them starts
    # meanwhile (a launch-bound call takes about this long per call whatever its kernels do)
    torch.cuda._sleep(int(2e9 * 0.02))
    t0 = time.perf_counter()
    for _ in range(min(reps, 10)):
        f()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{name} enqueue: {(t1 - t0) / min(reps, 10) * 1e3:.3f} ms per call", flush=True)
t0 = time.perf_counter()
for _ in range(reps):
    VrPlan(pat, P, light=True)
print(f"plan (light): {(time.perf_counter() - t0) / reps * 1e3:.3f} ms", flush=True)
