"""Config 4 host plan: rerun time with and without the control loop's transition stretches and
stretches through drops (FEC_VR_NO_FAST_TRANSITION, FEC_VR_NO_DROP_STRETCH, read per run),
alternating, best and median of N reruns each, plus a check that both give the same schedule.
  python tools/vr_plan_ab.py [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.vr import VrPlan  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
pat = load_pattern("bin_erasure")
P = 360000
w = VrPlan(pat, P, light=True)
res = {"fast": [], "slow": []}
ctl = {"fast": [], "slow": []}
for i in range(2 * reps):
    mode = "fast" if i % 2 else "slow"
    for k in ("FEC_VR_NO_FAST_TRANSITION", "FEC_VR_NO_DROP_STRETCH"):
        if mode == "slow":
            os.environ[k] = "1"
        else:
            os.environ.pop(k, None)
    t0 = time.perf_counter()
    w.rerun(pat, P, wait=True)
    res[mode].append((time.perf_counter() - t0) * 1e3)
    ctl[mode].append(w.plan_ms["control_loop"])
for m in ("slow", "fast"):
    r, c = sorted(res[m]), sorted(ctl[m])
    print(f"{m}: rerun best {r[0]:.3f} median {r[len(r) // 2]:.3f} ms; control loop best {c[0]:.3f} median "
          f"{c[len(c) // 2]:.3f} ms", flush=True)
os.environ["FEC_VR_NO_FAST_TRANSITION"] = os.environ["FEC_VR_NO_DROP_STRETCH"] = "1"
a = VrPlan(pat, P)
os.environ.pop("FEC_VR_NO_FAST_TRANSITION", None)
os.environ.pop("FEC_VR_NO_DROP_STRETCH", None)
b = VrPlan(pat, P)
same = all(np.array_equal(getattr(a, k), getattr(b, k)) for k in ("encoders", "decoders", "frames", "fate", "fate_decoder"))
print("schedules equal" if same else "schedules DIFFER", flush=True)
