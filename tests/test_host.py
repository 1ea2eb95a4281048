"""CPU checks of the product library: it loads, exports every declared entry point, and its
host-side control plane (decode rules + symbolic planner, the same algorithm the GPU's
fec_plan_kernel runs) reproduces the oracle's lost-packet sets.  No device work here."""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
from conftest import ROOT, load_pattern

import fec_erasure_code_unit_test_relay_amd as fec


def declared_functions(header):
    txt = open(header).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fec_[a-z_0-9]+)\s*\(", txt)))


def exported_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_library_loads_and_exports_c_abi():
    assert os.path.exists(fec.LIB_PATH)
    assert fec.lib().fec_version() == 2
    syms = exported_symbols(fec.LIB_PATH)
    names = declared_functions(os.path.join(ROOT, "include", "fec_amd.h"))
    assert len(names) >= 20
    missing = [n for n in names if n not in syms]
    assert not missing, missing


def test_library_exports_reference_named_cpp_api():
    syms = exported_symbols(fec.LIB_PATH)
    demangled = subprocess.run(["c++filt"], input="\n".join(sorted(syms)), capture_output=True,
                               text=True, check=True).stdout
    for sig in ["FEC_Encoder::FEC_Encoder(int, int, int, int, Memory_Allocator*)",
                "FEC_Encoder::onTransmit(unsigned char*, int, int, int*)",
                "FEC_Decoder::FEC_Decoder(int, int, int, int, Memory_Allocator*)",
                "FEC_Decoder::onReceive(unsigned char*, int, int, int*, bool)",
                "Memory_Allocator::allocate_memory(int)", "Encoder::getG()", "Decoder::getG()",
                "FEC_Message::set_parameters(int, int, int, int, int, unsigned char*)"]:
        assert sig in demangled, sig


def test_strerror_and_bad_arguments():
    assert fec.lib().fec_strerror(0) == b"ok"
    fate = np.zeros(4, dtype=np.uint8)
    er = np.zeros(4, dtype=np.uint8)
    import ctypes
    # B < N is rejected (every reference configuration has N <= B)
    st = fec.lib().fec_plan_host(300, 10, 1, 3, er.ctypes.data_as(ctypes.c_void_p), 4,
                                 fate.ctypes.data_as(ctypes.c_void_p))
    assert st == -1


def host_lost(T, B, N, pattern, P):
    pat = np.zeros(P + T, dtype=np.uint8)
    m = min(pattern.size, P + T)
    pat[:m] = pattern[:m]
    fate = fec.plan_host(300, T, B, N, pat)
    assert fate.size == P
    return fate


def test_planner_reproduces_published_loss_counts(published_runs):
    for run in published_runs:
        pat = load_pattern(run["pattern"])[:360000]
        fate = host_lost(run["T"], run["B"], run["N"], pat, 360000)
        assert int((fate == 3).sum()) == run["lost_packets"], run["log"]


def test_planner_matches_oracle_lost_lists(oracle_vectors):
    pat = load_pattern("bin_erasure")[:360000]
    for key, lost in oracle_vectors["lost"].items():
        T, B, N = map(int, key.split(","))
        fate = host_lost(T, B, N, pat, 360000)
        assert np.flatnonzero(fate == 3).tolist() == lost
        er = pat[:360000].astype(bool)
        assert ((fate == 1) == ~er).all()  # received packets are copied
        assert ((fate == 2) | (fate == 3))[er].all()


def bursty_pattern(rng, P, p_start, mean_burst, iid=0.0):
    pat = (rng.random(P) < iid).astype(np.uint8)
    t = 0
    while t < P:
        if rng.random() < p_start:
            b = 1 + rng.geometric(1.0 / mean_burst)
            pat[t:t + b] = 1
            t += b
        t += 1
    return pat


CONFIGS = [(10, 3, 3), (10, 5, 2), (10, 1, 1), (10, 0, 0), (10, 2, 2), (10, 5, 5), (10, 6, 6),
           (10, 7, 7), (10, 8, 8), (10, 9, 9), (10, 10, 10), (10, 3, 1), (10, 4, 3), (10, 5, 4),
           (10, 8, 4), (10, 9, 8), (5, 3, 1), (4, 6, 2), (3, 2, 2), (12, 4, 2)]


@pytest.mark.parametrize("tbn", CONFIGS)
def test_planner_matches_oracle_random_bursts(tbn):
    T, B, N = tbn
    rng = np.random.default_rng(abs(hash(tbn)) % 2**32)
    P = 6000
    pat = bursty_pattern(rng, P + T, 0.02, 3.0, iid=0.01)
    pat[:3] = 1  # startup erasures (NULL-slot replay)
    r = oracle.run_stream(300, T, B, N, P, pat, loss_only=True)
    fate = host_lost(T, B, N, pat, P)
    assert ((r["out_len"] == 0) == (fate == 3)).all()


@pytest.mark.parametrize("tbn", [(10, 9, 1), (10, 10, 1), (10, 8, 1), (10, 9, 2)])
def test_planner_without_rule_table_matches_oracle(tbn):
    """n = 18..21 (T = 10 allows it): no (window, mask) rule table, every rule computed on first
    use -- the planner still reproduces the oracle's lost list (restated gf256_rref_matrix per
    symbol, oracle/fec_oracle.c) packet for packet on the shipped erasure100 pattern."""
    T, B, N = tbn
    P = 30000
    pat = load_pattern("erasure100")[:P + T].astype(np.uint8)
    fate = host_lost(T, B, N, pat, P)
    ref = oracle.run_stream(300, T, B, N, P, pat, loss_only=True)
    assert (fate == 3).sum() > 0
    assert np.flatnonzero(fate == 3).tolist() == np.flatnonzero(ref["out_len"] == 0).tolist()
