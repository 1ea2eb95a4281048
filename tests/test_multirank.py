"""The N>1 path on CPU: world size 2 over gloo, the same partition and collectives bench.py uses over
RCCL (fec_erasure_code_unit_test_relay_amd/streams.py).

Each rank takes its own stream: payload seed 0x5EED+rank, and bin/erasure.bin replayed from phase
36000*rank. It plans the decode with the library's host planner (fec_plan_host, the control plane of
the product; no GPU needed) and checks the lost set against the oracle. Then the per-rank counters
are summed and the step times max-reduced, exactly as in bench.py. The parent process recomputes
every rank's stream on its own and compares the totals.
"""
import os
import socket

import numpy as np
import pytest

import oracle
from conftest import ROOT

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from fec_erasure_code_unit_test_relay_amd import plan_host  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import (load_pattern, max_over_ranks,  # noqa: E402
                                                          reduce_counters, stream_pattern,
                                                          stream_seed)

L, T, B, N = 300, 10, 3, 3
P = 4000


def _rank_stream(rank):
    pat = stream_pattern(P + T, rank, load_pattern("bin_erasure", ROOT))
    fate = plan_host(L, T, B, N, pat)
    lost = int((fate == 3).sum())
    ref = oracle.run_stream(L, T, B, N, P, pat, seed=stream_seed(rank), loss_only=True)
    ref_lost = ref["out_len"] == 0
    return pat, fate, lost, ref_lost


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pat, fate, lost, ref_lost = _rank_stream(rank)
        agree = bool(((fate == 3) == ref_lost).all())
        totals = reduce_counters([lost, int(pat[:P].sum()), int(agree)], dist)
        t = max_over_ranks(0.25 * (rank + 1), dist)
        dist.barrier()
        q.put((rank, totals, t))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_streams_are_independent_and_distinct():
    base = load_pattern("bin_erasure", ROOT)
    p0 = stream_pattern(P + T, 0, base)
    p1 = stream_pattern(P + T, 1, base)
    assert (p0 == base[: P + T]).all()
    assert (p1 == base[36000: 36000 + P + T]).all()
    assert not (p0 == p1).all()
    # replay wraps at 360000 packets
    long = stream_pattern(360000 + 50, 0, base)
    assert (long[360000:] == base[:50]).all()
    assert stream_seed(0) != stream_seed(1)


def test_two_ranks_gloo_partition_and_reduction():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp_lost = exp_erased = 0
    for r in range(world):
        pat, fate, lost, ref_lost = _rank_stream(r)
        assert ((fate == 3) == ref_lost).all()
        exp_lost += lost
        exp_erased += int(pat[:P].sum())
    for rank, totals, t in results:
        assert totals == [exp_lost, exp_erased, world], (rank, totals)
        assert t == pytest.approx(0.25 * world)
    assert np.isfinite(exp_lost) and exp_erased > 0
