"""Bench step with the batch cut into NC chunks: the encoder of chunk i+1 runs beside the copy of
chunk i (two streams), the plan beside both, the recovery after everything.  Outputs are checked
against the one-shot step; times are graph-replayed steps, same process, same buffers.
  python tools/overlap_exp.py 1 2 4 8"""
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
plan_after = int(os.environ.get("PLAN_AFTER", "1"))  # plan starts after encoder chunk #k (0: at once)


def base_step():
    c.encode(payload, out=cw, out_len=wl)
    c.decode(cw, er, out=out, out_len=ol)


s_copy, s_plan = torch.cuda.Stream(), torch.cuda.Stream()


def chunked(nc):
    cuts = [P * i // nc for i in range(nc + 1)]

    def step():
        cur = torch.cuda.current_stream()
        s_copy.wait_stream(cur)
        s_plan.wait_stream(cur)
        for i in range(nc):
            a, b = cuts[i], cuts[i + 1]
            bb = Pf if i == nc - 1 else b
            h = min(a, c.n - 1)
            c.encode(payload[a - h:bb], history=h, out=cw[a:bb], out_len=wl[a:bb])
            ev = torch.cuda.Event()
            ev.record()
            if i + 1 == plan_after or (plan_after == 0 and i == 0):
                s_plan.wait_event(ev) if plan_after else None
                with torch.cuda.stream(s_plan):
                    c.plan(er, Pf)
            with torch.cuda.stream(s_copy):
                s_copy.wait_event(ev)
                c.copy(cw[a:b + T], er[a:b + T], out=out[a:b], out_len=ol[a:b])
        cur.wait_stream(s_copy)
        cur.wait_stream(s_plan)
        c.recover(cw, out, ol)
    return step


def graphed(fn):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g.replay


base_step()
torch.cuda.synchronize()
ref_out, ref_ol = out.clone(), ol.clone()
variants = {"oneshot": graphed(base_step)}
for a in sys.argv[1:]:
    nc = int(a)
    fn = chunked(nc)
    out.zero_()
    ol.fill_(-1)
    fn()
    torch.cuda.synchronize()
    assert torch.equal(out, ref_out) and torch.equal(ol, ref_ol), f"chunked {nc} differs"
    variants[f"chunks{nc}"] = graphed(fn)
t_end = time.perf_counter() + 1.0
while time.perf_counter() < t_end:
    for f in variants.values():
        f()
    torch.cuda.synchronize()
res = {k: [] for k in variants}
for rnd in range(7):
    for k, f in variants.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            f()
        torch.cuda.synchronize()
        res[k].append((time.perf_counter() - t0) / 20 * 1e3)
print(f"PLAN_AFTER={plan_after}  " + "  ".join(f"{k}: {sorted(v)[3]:.4f} ms ({P * L / sorted(v)[3] / 1e-3 / 2**30:.1f} GiB/s)"
                for k, v in res.items()), flush=True)
