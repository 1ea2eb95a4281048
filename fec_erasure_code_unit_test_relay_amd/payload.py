"""Synthetic 300-byte payloads generated on the GPU (tests and bench.py only).

Byte b of packet t = splitmix64(seed ^ (t*L + b)) & 0xff, identical to oracle/fec_oracle.c's
or_fill_payload, so that device-generated inputs can be checked against the CPU restatement.
"""
from __future__ import annotations

import ctypes

from ._lib import check, lib


def fill_payload(t0: int, count: int, L: int, seed: int = 0x5EED, device="cuda", out=None):
    import torch
    if out is None:
        out = torch.empty((count, L), dtype=torch.uint8, device=device)
    check(lib().fec_util_fill_payload(ctypes.c_void_p(out.data_ptr()), t0, count, L,
                                      ctypes.c_uint64(seed),
                                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
          "fec_util_fill_payload")
    return out
