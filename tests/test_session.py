"""The two-hop adaptive relay session (RELAYING_TYPE 2 / 3 with N_INITIAL = N_INITIAL_2 = -1,
application_local_simulation.cpp:71-593): the oracle's reference-structured loop
(or_relay_session_run, oracle/fec_oracle.c) on its own -- hand-checked properties of the
reference's control flow -- and against the committed 360 000-seq digests (parity unpinned: the
reference ships no relay output; tests/golden/relay_session_360k.json comes from this oracle,
tests/golden/make_relay_session_golden.py).  The GPU session is checked against both in
tests/test_gpu_session.py."""
import json
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, load_pattern

Q_SMALL = 3000


def _run(R, Q, e1, e2, **kw):
    return oracle.relay_session_run(R, Q, e1, e2, want_out=True, **kw)


@pytest.mark.parametrize("R", [2, 3])
def test_clean_channel_loses_nothing(R):
    z = np.zeros(Q_SMALL, np.uint8)
    r = _run(R, Q_SMALL, z, z)
    assert r["lost"] == 0 and r["dest_proc"].sum() == Q_SMALL and r["src_switches"] == 0
    # the source never leaves (T_TOT, 0, 0): every hop-1 header says T = 10, N = 0, T2 = 10
    assert (r["hop1_hdr"][:, 4] == 10).all() and (r["hop1_hdr"][:, 6] == 0).all()
    assert (r["hop1_hdr"][:, 8] == 10).all()
    # the relay sends n2 = T2 + 1 = 11, k2 = 11 (N2 = 0) and the destination outputs packet t - T_TOT
    assert (r["relay_hdr"][:, 4] == 10).all() and (r["relay_hdr"][:, 6] == 0).all()
    pay = oracle.fill_payload(0, Q_SMALL - 10, 300, 0x5EED)
    out = r["dest_out"][10:, 2:302]
    assert np.array_equal(out, pay)


@pytest.mark.parametrize("R", [2, 3])
def test_hop1_burst_then_adaptation(R):
    """A 3-packet hop-1 burst on an uncoded first hop: the three packets are lost at the destination
    (T_TOT = 10 seqs later), the relay's estimate (N = 3) reaches the source with the 12-byte
    feedback, the source splits T_TOT (T = T_TOT - N2 = 10, T2 = T_TOT - N = 7) and switches."""
    z = np.zeros(Q_SMALL, np.uint8)
    e1 = z.copy()
    e1[500:503] = 1
    r = _run(R, Q_SMALL, e1, z)
    assert r["lost"] == 3 and list(np.nonzero(r["dest_lost"])[0]) == [510, 511, 512]
    h = r["hop1_hdr"].astype(int)
    sw = np.nonzero((h[1:, 4] != h[:-1, 4]) | (h[1:, 6] != h[:-1, 6]))[0] + 1
    assert len(sw) >= 1
    s = sw[0]
    assert h[s, 7] == 0 and h[s, 11] == 0                        # counter restarts at the switch
    assert h[s, 4] - h[s, 6] + 1 == h[s, 8] - h[s, 10] + 1       # k == k2 across the split
    assert h[s, 8] == 10 - h[s, 6]                               # T2 = T_TOT - N
    assert h[s, 12] == h[s - 1, 4] and h[s, 13] == h[s - 1, 6]   # T_old, N_old
    # double coding: T_TOT + 1 packets carry two codewords
    L1 = r["hop1_len"]
    assert (L1[s:s + 11] > L1[s + 11:s + 20].max()).all()
    # hand-traced relay word layout through the switch (Variable_Rate_FEC_Decoder.cpp:1458-1588,
    # send_sym_wise_message :317-330): [8-byte header][size_cur BE16][new part][old part] during the
    # relay's double coding (seqs s .. s + T_TOT), one part before and after; a part is
    # codeword_r_d_size = (ceil(302 / k2) + 1) * n2 bytes (:997-999), plus its 11-byte header row
    # for type 3; the 8-byte header carries the new hop-2 code (n2 - 1, n2 - k2, n2 - k2)
    def rd(k2, n2):
        return (-(-302 // k2) + 1) * n2
    hb = 11 if R == 3 else 0
    k_old, n2_old = h[s - 1, 8] - h[s - 1, 10] + 1, h[s - 1, 8] + 1   # (11, 11) before the switch
    k_new, n2_new = h[s, 8] - h[s, 10] + 1, h[s, 8] + 1
    RL, RH = r["relay_len"], r["relay_hdr"].astype(int)
    assert RL[s - 1] == 8 + 2 + hb + rd(k_old, n2_old)
    for t in range(s, s + 11):
        assert RL[t] == 8 + 2 + hb + rd(k_new, n2_new) + hb + rd(k_old, n2_old)
        assert RH[t, 4] == n2_new - 1 and RH[t, 6] == n2_new - k_new
    assert RL[s + 11] == 8 + 2 + hb + rd(k_new, n2_new)


@pytest.mark.parametrize("R", [2, 3])
def test_hop2_burst_reaches_the_source(R):
    """A hop-2 burst: the destination's 6-byte feedback rides in bytes 6..11 of the relay's 12-byte
    response, so the source raises N2 and shortens its own T (T = T_TOT - N2)."""
    z = np.zeros(Q_SMALL, np.uint8)
    e2 = z.copy()
    e2[500:503] = 1
    r = _run(R, Q_SMALL, z, e2)
    h = r["hop1_hdr"].astype(int)
    after = h[600:]
    assert (after[:, 10] > 0).any()                 # N2 > 0 announced
    i = np.nonzero(after[:, 10] > 0)[0][0]
    assert after[i, 4] == 10 - after[i, 10]         # T = T_TOT - N2 once the switch happens
    assert r["lost"] >= 3


@pytest.mark.parametrize("R", [2, 3])
def test_session_on_shipped_patterns_is_deterministic(R):
    e1, e2 = load_pattern("bin_erasure"), load_pattern("bin_erasure2")
    a = _run(R, Q_SMALL, e1, e2)
    b = _run(R, Q_SMALL, e1, e2)
    assert np.array_equal(a["crc"], b["crc"]) and np.array_equal(a["crc2"], b["crc2"])
    assert a["lost"] == b["lost"] and a["src_switches"] > 10
    # every received frame's processed flag: the destination outputs every seq it reaches
    assert a["dest_proc"][: Q_SMALL - 20].all()


def test_session_golden_prefix():
    """The first blocks of the committed 360 000-seq digests re-derived (type 2, fast enough here)."""
    g = json.load(open(os.path.join(GOLDEN, "relay_session_360k.json")))
    e1, e2 = load_pattern("bin_erasure"), load_pattern("bin_erasure2")
    n = 30
    r = _run(2, n * oracle.SESSION_BLOCK, e1, e2)
    ref = g["types"]["2"]
    assert [int(x) for x in r["crc"][:n]] == ref["crc"][:n]
    # a seq's destination output can come after the last seq of a shorter run: the last block waits
    assert [int(x) for x in r["crc2"][:n - 1]] == ref["crc2"][:n - 1]
