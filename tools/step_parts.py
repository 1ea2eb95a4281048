"""Event-timed parts of the bench step in one process (same buffers):
encode alone, plan alone, copy alone, copy beside the plan, recover, whole eager step.
  python tools/step_parts.py [--packets 1000000] [--tbn 10,3,3]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import L, stream_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--packets", type=int, default=1_000_000)
ap.add_argument("--tbn", default="10,3,3")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--grids", default="", help="FEC_PLAN_GRID values to sweep, e.g. 8192,1024,256")
args = ap.parse_args()
T, B, N = map(int, args.tbn.split(","))
torch.cuda.set_device(0)
P = args.packets
Pf = P + T
c = Codec(L, T, B, N)
payload = fill_payload(0, Pf, L, 0x5EED)
er = torch.from_numpy(stream_pattern(Pf, 0)).cuda()
cw = torch.empty((Pf, c.CW), dtype=torch.uint8, device="cuda")
wl = torch.empty(Pf, dtype=torch.int32, device="cuda")
out = torch.empty((P, L), dtype=torch.uint8, device="cuda")
ol = torch.empty(P, dtype=torch.int32, device="cuda")
c.workspace(Pf)
side = torch.cuda.Stream()
main = torch.cuda.Stream()  # not the null stream: a blocking side stream would sync with it
torch.cuda.set_stream(main)


def timed(fn, reps=args.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def enc():
    c.encode(payload, out=cw, out_len=wl)


def plan():
    c.plan(er)


def copy():
    c.copy(cw, er, out=out, out_len=ol)


def copy_beside_plan():
    fork = torch.cuda.Event()
    fork.record()
    with torch.cuda.stream(side):
        side.wait_event(fork)
        c.plan(er)
    c.copy(cw, er, out=out, out_len=ol)
    main.wait_stream(side)


def overlap_detail(reps=10):
    """copy on the main stream beside the plan on the side stream: each one's own event time"""
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    res = []
    for _ in range(reps + 1):
        fork = torch.cuda.Event()
        fork.record()
        with torch.cuda.stream(side):
            side.wait_event(fork)
            ev[2].record(side)
            c.plan(er)
            ev[3].record(side)
        ev[0].record()
        c.copy(cw, er, out=out, out_len=ol)
        ev[1].record()
        main.wait_stream(side)
        torch.cuda.synchronize()
        res.append((ev[0].elapsed_time(ev[1]) * 1e3, ev[2].elapsed_time(ev[3]) * 1e3,
                    ev[0].elapsed_time(ev[2]) * 1e3, ev[0].elapsed_time(ev[3]) * 1e3))
    res = sorted(res[1:])
    return res[len(res) // 2]


def recover():
    c.recover(cw, out, ol)


def dec():
    c.decode(cw, er, out=out, out_len=ol)


def step():
    enc()
    dec()


res = {}
for rnd in range(3):
    for name, fn in [("encode", enc), ("plan", plan), ("copy", copy), ("copy||plan", copy_beside_plan),
                     ("recover", recover), ("decode", dec), ("step", step)]:
        res.setdefault(name, []).append(timed(fn))
print(f"P={P} tbn={args.tbn} " + "  ".join(f"{k}: {sorted(v)[1]:.1f} us" for k, v in res.items()), flush=True)
print("plan_stats (replayed, duplicates)", c.plan_stats(), flush=True)
cp, pl, ps, pe = overlap_detail()
print(f"  beside each other: copy {cp:.1f} us, plan {pl:.1f} us; from the copy's start: plan starts "
      f"{ps:.1f}, ends {pe:.1f} us", flush=True)
os.environ["FEC_PLAN_GRID"] = "256"
cp, pl, ps, pe = overlap_detail()
print(f"  (plan grid 256) beside each other: copy {cp:.1f} us, plan {pl:.1f} us; from the copy's start: plan starts "
      f"{ps:.1f}, ends {pe:.1f} us", flush=True)
os.environ.pop("FEC_PLAN_GRID")
if args.grids:
    for g in args.grids.split(","):
        os.environ["FEC_PLAN_GRID"] = g
        r = {name: timed(fn) for name, fn in [("plan", plan), ("copy||plan", copy_beside_plan), ("step", step)]}
        print(f"  FEC_PLAN_GRID={g}: " + "  ".join(f"{k}: {v:.1f} us" for k, v in r.items()), flush=True)
    os.environ.pop("FEC_PLAN_GRID")
dec()
torch.cuda.synchronize()
assert torch.equal(out[ol != 0], payload[:P][ol != 0])
print("counters", c.counters(), flush=True)
