"""Config 4 host plan A/B on the box host: the plan from scratch (fec_vr_plan_rerun, waited for) under
environment variants, interleaved, on the least busy 8-CPU group (as bench.py's config 4).
    python tools/vr_plan_ab.py [rounds]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import quiet_cpu_group  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.vr import VrPlan  # noqa: E402

VARIANTS = {
    "default": {},
    "fb_stop (round 5 steady stretches)": {"FEC_VR_FB_STOP": "1"},
    "fb job per queue entry (r06d)": {"FEC_VR_FB_CHUNKS": "100000"},
    "fb producer thread (round 5)": {"FEC_VR_FB_THREAD": "1"},
    "fb_stop + producer thread (r06c)": {"FEC_VR_FB_STOP": "1", "FEC_VR_FB_THREAD": "1"},
}
KEYS = [k for v in VARIANTS.values() for k in v]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    pat = load_pattern("bin_erasure")
    P = 360000
    group = quiet_cpu_group()
    if group:
        os.sched_setaffinity(0, group)
    w = VrPlan(pat, P, light=True)
    res = {n: [] for n in VARIANTS}
    for _ in range(rounds):
        for name, env in VARIANTS.items():
            for k in KEYS:
                os.environ.pop(k, None)
            os.environ.update(env)
            for _ in range(10):
                res[name].append(w.rerun(pat, P, wait=True).plan_ms)
    for k in KEYS:
        os.environ.pop(k, None)
    print(f"cpu group {group[0]}-{group[-1]}" if group else "cpu group: none")
    for name, runs in res.items():
        tot = [r["control_loop"] + r["decoder_instances"] for r in runs]
        med = {k: float(np.median([r[k] for r in runs])) for k in runs[0]}
        print(f"{name:40s} plan median {np.median(tot):.3f} ms (min {min(tot):.3f}) | " +
              " ".join(f"{k} {v:.3f}" for k, v in med.items()))


if __name__ == "__main__":
    main()
