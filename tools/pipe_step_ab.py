"""Sequential bench steps vs steps software-pipelined across batches (encode of batch i+1 on one stream
while batch i is decoded on another, codewords and outputs double-buffered), one process, alternating
rounds; outputs compared.   python tools/pipe_step_ab.py [rounds]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import L, stream_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload  # noqa: E402

torch.cuda.set_device(0)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
P, T = 1_000_000, 10
Pf = P + T
c = Codec(L, 10, 3, 3)
payload = fill_payload(0, Pf, L, 0x5EED)
er = torch.from_numpy(stream_pattern(Pf, 0)).cuda()
cw = [torch.empty((Pf, c.CW), dtype=torch.uint8, device="cuda") for _ in range(2)]
wl = [torch.empty(Pf, dtype=torch.int32, device="cuda") for _ in range(2)]
out = [torch.empty((P, L), dtype=torch.uint8, device="cuda") for _ in range(2)]
ol = [torch.empty(P, dtype=torch.int32, device="cuda") for _ in range(2)]
c.workspace(Pf)
sE, sD = torch.cuda.Stream(), torch.cuda.Stream()
ev_enc = [torch.cuda.Event() for _ in range(2)]
ev_dec = [torch.cuda.Event() for _ in range(2)]
cnt = [0]


def seq_step():
    c.encode(payload, out=cw[0], out_len=wl[0])
    c.decode(cw[0], er, out=out[0], out_len=ol[0])


def pipe_step():
    i = cnt[0]
    cnt[0] += 1
    b = i & 1
    with torch.cuda.stream(sE):
        if i >= 2:
            sE.wait_event(ev_dec[b])
        c.encode(payload, out=cw[b], out_len=wl[b])
        ev_enc[b].record(sE)
    with torch.cuda.stream(sD):
        sD.wait_event(ev_enc[b])
        c.decode(cw[b], er, out=out[b], out_len=ol[b])
        ev_dec[b].record(sD)


sP = torch.cuda.Stream()
ev_copy = [torch.cuda.Event() for _ in range(2)]
ev_rec = [torch.cuda.Event() for _ in range(2)]
ev_plan = [torch.cuda.Event() for _ in range(2)]


def pipe2_step():
    """The next batch's encode starts when this batch's copy ends: it overlaps the recovery and the
    launch gaps only (the plan still runs beside the copy)."""
    i = cnt[0]
    cnt[0] += 1
    b = i & 1
    with torch.cuda.stream(sE):
        if i >= 1:
            sE.wait_event(ev_copy[b ^ 1])
        c.encode(payload, out=cw[b], out_len=wl[b])
        ev_enc[b].record(sE)
    with torch.cuda.stream(sP):
        sP.wait_event(ev_enc[b])
        if i >= 1:
            sP.wait_event(ev_rec[b ^ 1])
        c.plan(er)
        ev_plan[b].record(sP)
    with torch.cuda.stream(sD):
        sD.wait_event(ev_enc[b])
        c.copy(cw[b], er, out=out[b], out_len=ol[b])
        ev_copy[b].record(sD)
        sD.wait_event(ev_plan[b])
        c.recover(cw[b], out=out[b], out_len=ol[b])
        ev_rec[b].record(sD)


def run(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for fn in (seq_step, pipe_step, pipe2_step):
    cnt[0] = 0
    run(fn, 300)
ref = (out[0].clone(), ol[0].clone())
res = {"seq": [], "pipe": [], "pipe2": []}
outs = {}
for r in range(rounds):
    res["seq"].append(run(seq_step, 100))
    for name, fn in (("pipe", pipe_step), ("pipe2", pipe2_step)):
        cnt[0] = 0  # the pipeline restarts after a full synchronisation
        res[name].append(run(fn, 100))
        outs[name] = all(torch.equal(out[b], ref[0]) and torch.equal(ol[b], ref[1]) for b in range(2))
for k, v in res.items():
    v = sorted(v)
    print(f"{k}: step median {v[len(v) // 2]:.4f} ms, best {v[0]:.4f} ms", flush=True)
print("outputs equal" if all(outs.values()) else f"outputs DIFFER {outs}", flush=True)
