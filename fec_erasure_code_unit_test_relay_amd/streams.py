"""Multi-GPU partition of the workload: one independent packet stream per rank.

Streams share nothing: each rank encodes its own payloads (seed + rank) and decodes them under its
own erasure phase. The only collectives are around the data path: a barrier before and after the
timed region, the max-over-ranks step time, and one sum of the per-rank counters. On ROCm these go
over RCCL ("nccl" backend) and over xGMI; the tests run the same code over gloo on the CPU.
"""
from __future__ import annotations

import os

import numpy as np

PAYLOAD_SEED = 0x5EED
PATTERN_PERIOD = 360000     # packets of bin/erasure.bin that are replayed
PATTERN_PHASE = 36000       # per-rank phase offset into the replayed pattern


def load_pattern(name: str = "bin_erasure", root: str | None = None) -> np.ndarray:
    """A shipped erasure pattern (one byte per packet, 1 = erased) from tests/golden."""
    root = root or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    z = np.load(os.path.join(root, "tests", "golden", "erasure_patterns.npz"))
    return np.unpackbits(z[name])[: int(z[name + "_len"][0])].astype(np.uint8)


def stream_seed(rank: int) -> int:
    """Payload seed of rank's stream."""
    return PAYLOAD_SEED + rank


def stream_pattern(P_fed: int, rank: int, base: np.ndarray | None = None) -> np.ndarray:
    """Erasure flags of rank's stream: bin/erasure.bin's first 360000 packets replayed cyclically,
    starting at phase 36000*rank (ERASURE_TYPE=5 replay semantics, Erasure_Simulator.cpp:53)."""
    if base is None:
        base = load_pattern("bin_erasure")
    base = base[:PATTERN_PERIOD]
    shift = (PATTERN_PHASE * rank) % base.size
    reps = -(-(P_fed + shift) // base.size)
    return np.tile(base, reps)[shift: shift + P_fed].copy()


def reduce_counters(values, dist=None, device=None):
    """Sum integer counters over all ranks (a no-op without an initialised process group)."""
    import torch
    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
    return [int(x) for x in t.tolist()]


def max_over_ranks(seconds: float, dist=None, device=None) -> float:
    """The slowest rank's time (the job's time under weak scaling)."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
