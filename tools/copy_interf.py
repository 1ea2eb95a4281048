"""Copy kernel alone vs beside the planner (and parts of it: FEC_PLAN_SKIP)."""
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
c = Codec(L, 10, 3, 3)
payload = fill_payload(0, Pf, L, 0x5EED)
er = torch.from_numpy(stream_pattern(Pf, 0)).cuda()
cw, wl = c.encode(payload)
out = torch.empty((P, L), dtype=torch.uint8, device="cuda")
ol = torch.empty(P, dtype=torch.int32, device="cuda")
c.workspace(Pf)
side = torch.cuda.Stream()
main = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def run(with_plan):
    fork = torch.cuda.Event()
    fork.record()
    if with_plan:
        with torch.cuda.stream(side):
            side.wait_event(fork)
            c.plan(er)
    e0.record()
    c.copy(cw, er, out=out, out_len=ol)
    e1.record()
    main.wait_stream(side)


res = {}
for rnd in range(5):
    for cfg in ["alone", "plan", "skip1", "skip2", "skip4", "skip7"]:
        os.environ["FEC_PLAN_SKIP"] = cfg[4:] if cfg.startswith("skip") else "0"
        run(cfg != "alone")
        torch.cuda.synchronize()
        t = []
        for _ in range(10):
            run(cfg != "alone")
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1) * 1e3)
        res.setdefault(cfg, []).append(sorted(t)[5])
print("  ".join(f"{k}: {sorted(v)[2]:.1f} us" for k, v in res.items()))
