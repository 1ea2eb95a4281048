"""Erasure patterns: the inputs of the decode path, mirroring the reference's
Erasure_File_Generator (src/Erasure_File_Generator.cpp) and Erasure_Simulator
(src/Erasure_Simulator.cpp) with the same method names and arguments.

The generators run in the C++ host code of libfec_amd.so (fec_erasure.cpp: mt19937 and libstdc++'s
uniform_real_distribution<double> arithmetic restated), byte-exact with the reference: the
shipped bin/erasure.bin and bin/erasure2.bin are generate_Fritchman_varying(360010, ALPHA, BETA,
1e-4, NUMBER_OF_STATES, ..., seed 0 / 1) (tests/test_erasure.py).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib

# include/FEC_Macro.h:80-100
SEED_ARTIFICIAL_ERASURE = 0
ALPHA = 0.005
BETA = 0.990
NUMBER_OF_STATES = 6


def _buf(count: int) -> tuple[np.ndarray, ctypes.c_void_p]:
    if count < 0:
        raise ValueError("count < 0")
    out = np.zeros(max(count, 1), dtype=np.uint8)
    return out, out.ctypes.data_as(ctypes.c_void_p)


class Erasure_File_Generator:
    """Same interface as the reference class (include/Erasure_File_Generator.h).  Every generator
    returns the pattern (uint8, 1 = erased) and, when `filename` is given, writes it as the
    reference does (one byte per packet).  The Gilbert-Elliott generators carry `good_state`
    across calls on the same object, as the reference's member does."""

    def __init__(self) -> None:
        self.good_state = True

    @staticmethod
    def _finish(out: np.ndarray, count: int, filename: str | None) -> np.ndarray:
        out = out[:count]
        if filename:
            out.tofile(filename)
        return out

    def generate_IID(self, number_of_erasure: int, erasure_prob: float, filename: str | None = None,
                     seed: int = 0) -> np.ndarray:
        out, p = _buf(number_of_erasure)
        check(lib().fec_erasure_iid(p, number_of_erasure, erasure_prob, seed), "fec_erasure_iid")
        return self._finish(out, number_of_erasure, filename)

    def generate_three_sections_IID(self, n1: int, p1: float, n2: int, p2: float, n3: int, p3: float,
                                    filename: str | None = None, seed: int = 0) -> np.ndarray:
        out, p = _buf(n1 + n2 + n3)
        check(lib().fec_erasure_three_sections_iid(p, n1, p1, n2, p2, n3, p3, seed),
              "fec_erasure_three_sections_iid")
        return self._finish(out, n1 + n2 + n3, filename)

    def _ge(self, fn, number_of_erasure, alpha, beta, erasure_prob, filename, seed):
        out, p = _buf(number_of_erasure)
        st = ctypes.c_int(1 if self.good_state else 0)
        check(fn(p, number_of_erasure, alpha, beta, erasure_prob, seed, ctypes.byref(st)), fn.__name__)
        self.good_state = bool(st.value)
        return self._finish(out, number_of_erasure, filename)

    def generate_GE(self, number_of_erasure: int, alpha: float, beta: float, erasure_prob: float,
                    filename: str | None = None, seed: int = 0) -> np.ndarray:
        return self._ge(lib().fec_erasure_ge, number_of_erasure, alpha, beta, erasure_prob, filename, seed)

    def generate_GE_varying(self, number_of_erasure: int, alpha: float, beta: float, erasure_prob: float,
                            filename: str | None = None, seed: int = 0) -> np.ndarray:
        return self._ge(lib().fec_erasure_ge_varying, number_of_erasure, alpha, beta, erasure_prob,
                        filename, seed)

    def generate_Fritchman_varying(self, number_of_erasure: int, alpha: float, beta: float,
                                   erasure_prob: float, number_of_states: int,
                                   filename: str | None = None, seed: int = 0) -> np.ndarray:
        out, p = _buf(number_of_erasure)
        check(lib().fec_erasure_fritchman_varying(p, number_of_erasure, alpha, beta, erasure_prob,
                                                  number_of_states, seed), "fec_erasure_fritchman_varying")
        return self._finish(out, number_of_erasure, filename)

    def generate_periodic(self, number_of_erasure: int, T: int, B: int, N: int,
                          filename: str | None = None) -> np.ndarray:
        out, p = _buf(number_of_erasure)
        check(lib().fec_erasure_periodic(p, number_of_erasure, T, B, N), "fec_erasure_periodic")
        return self._finish(out, number_of_erasure, filename)


class Erasure_Simulator:
    """Replays an erasure pattern (ERASURE_TYPE 5): src/Erasure_Simulator.cpp:13-56.  Built from a
    file (one byte per packet) or an array; the no-argument form is the reference's built-in
    10000-packet pattern (:32-45).  Past the pattern's end every packet counts as received (the
    reference reads out of bounds there)."""

    def __init__(self, source: str | np.ndarray | None = None) -> None:
        if source is None:
            seq = np.arange(10000)
            self.erasure_seq = (((seq >= 5) & (seq <= 8)) | ((seq >= 16) & (seq <= 19)) |
                                ((seq >= 27) & (seq <= 30)) | ((seq >= 38) & (seq <= 41))).astype(np.uint8)
        elif isinstance(source, str):
            self.erasure_seq = np.fromfile(source, dtype=np.uint8)
        else:
            self.erasure_seq = np.ascontiguousarray(source, dtype=np.uint8)
        self.number_of_erasure = int(self.erasure_seq.size)

    def is_erasure(self, seq: int) -> bool:
        return 0 <= seq < self.number_of_erasure and self.erasure_seq[seq] == 1

    def pattern(self, count: int, start: int = 0) -> np.ndarray:
        """erasure flags of packets start .. start+count-1 (the batched decoder's input)"""
        out = np.zeros(count, dtype=np.uint8)
        lo, hi = max(start, 0), min(start + count, self.number_of_erasure)
        if hi > lo:
            out[lo - start:hi - start] = self.erasure_seq[lo:hi] == 1
        return out
