"""The oracle (CPU restatement, oracle/) checked against the reference's own published results.

Runs on CPU only.  Pins: 12 published fixed-rate loss counts (Experimental_Logs), ISA-L's field
definition, the survey's Cauchy entries, and self-consistency (every recovered payload equals its
source; the closed-form encoder used by the GPU kernel equals the reference-structured encoder).
"""
import hashlib

import numpy as np
import pytest

import oracle
from conftest import load_pattern


def clmul_mod(a: int, b: int) -> int:
    r = 0
    for i in range(8):
        if (b >> i) & 1:
            r ^= a << i
    for bit in range(14, 7, -1):
        if (r >> bit) & 1:
            r ^= 0x11D << (bit - 8)
    return r


def test_field_is_isal_gf256():
    rng = np.random.default_rng(1)
    pairs = [(a, b) for a in range(256) for b in (0, 1, 2, 3, 0x1D, 0x80, 0xFF)]
    pairs += [tuple(x) for x in rng.integers(0, 256, size=(3000, 2))]
    for a, b in pairs:
        assert oracle.gf_mul(int(a), int(b)) == clmul_mod(int(a), int(b))
    for a in range(1, 256):
        assert oracle.gf_mul(a, oracle.gf_inv(a)) == 1
    assert oracle.gf_inv(0) == 0


def test_generator_known_entries():
    G = oracle.gen_G(10, 3, 3)
    assert G.shape == (8, 11)
    assert (G[:, :8] == np.eye(8, dtype=np.uint8)).all()
    assert G[0, 8:].tolist() == [173, 157, 221]  # inv(8), inv(9), inv(10)
    for i in range(8):
        for j in range(8, 11):
            assert G[i, j] == oracle.gf_inv(i ^ j)
    # the RS special case (codingOperations.cpp:53-56)
    Grs = oracle.gen_G(10, 8, 4)
    k = 7
    assert (Grs[:, :k] == np.eye(k, dtype=np.uint8)).all()


@pytest.mark.parametrize("idx", range(12))
def test_published_fixed_rate_loss_counts(idx, published_runs):
    run = published_runs[idx]
    pat = load_pattern(run["pattern"])[:360000]
    assert int(pat.sum()) == run["udp_lost_packets"]
    r = oracle.run_stream(300, run["T"], run["B"], run["N"], 360000, pat, loss_only=True)
    assert r["lost"] == run["lost_packets"], run["log"]


def test_survey_loss_lists(oracle_vectors):
    pat = load_pattern("bin_erasure")[:360000]
    for key, lost in oracle_vectors["lost"].items():
        T, B, N = map(int, key.split(","))
        r = oracle.run_stream(300, T, B, N, 360000, pat, loss_only=True)
        assert np.flatnonzero(r["out_len"] == 0).tolist() == lost
    assert len(oracle_vectors["lost"]["10,5,2"]) == 565
    assert len(oracle_vectors["lost"]["10,3,3"]) == 4662


def test_loss_only_mode_matches_full_mode():
    pat = load_pattern("erasure100")[:3000]
    full = oracle.run_stream(300, 10, 9, 8, 3000, pat, want_data=True)
    lo = oracle.run_stream(300, 10, 9, 8, 3000, pat, loss_only=True)
    assert ((full["out_len"] == 0) == (lo["out_len"] == 0)).all()


@pytest.mark.parametrize("tbn,pattern,P", [((10, 5, 2), "bin_erasure", 6000),
                                           ((10, 9, 8), "erasure100", 2500),
                                           ((10, 10, 10), "erasure90", 1500)])
def test_recovered_payloads_equal_source(tbn, pattern, P):
    pat = load_pattern(pattern)[:P]
    r = oracle.run_stream(300, *tbn, P, pat, want_data=True)
    src = oracle.fill_payload(0, P, 300, 0x5EED)
    ok = r["out_len"] > 0
    assert ok.sum() > 0 and (r["out_len"][ok] == 300).all()
    assert (r["out_data"][ok] == src[ok]).all()
    assert (r["out_data"][~ok] == 0).all()


def closed_form_encode(G, payload, lens, k, n, S, L):
    """cw_t[s*n+j] = X_t[s][j] (j<k); XOR_i G[i][j] * X_{t-(j-i)}[s][i] (j>=k)."""
    P = payload.shape[0]
    X = np.zeros((P, S * k), dtype=np.uint8)
    for t in range(P):
        ln = lens[t]
        X[t, 0], X[t, 1] = ln >> 8, ln & 0xFF
        X[t, 2:2 + ln] = payload[t, :ln]
    X = X.reshape(P, S, k)
    mul = np.array([[oracle.gf_mul(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)
    cw = np.zeros((P, S, n), dtype=np.uint8)
    cw[:, :, :k] = X
    for j in range(k, n):
        acc = np.zeros((P, S), dtype=np.uint8)
        for i in range(k):
            d = j - i
            sh = np.zeros((P, S), dtype=np.uint8)
            sh[d:] = X[:P - d, :, i]
            acc ^= mul[G[i, j]][sh]
        cw[:, :, j] = acc
    return cw.reshape(P, S * n)


@pytest.mark.parametrize("tbn", [(10, 3, 3), (10, 5, 2), (10, 1, 1), (10, 0, 0), (10, 10, 10),
                                 (10, 9, 9), (10, 8, 4), (10, 5, 4), (10, 9, 8), (4, 6, 2)])
def test_closed_form_encoder_equals_structured_encoder(tbn):
    T, B, N = tbn
    k, n, S, CW = oracle.geometry(300, T, B, N)
    P = 400
    rng = np.random.default_rng(sum(tbn))
    payload = oracle.fill_payload(0, P, 300, 7)
    lens = rng.integers(0, 301, size=P)
    lens[:50] = 300
    enc = oracle.Encoder(300, T, B, N)
    ref = np.zeros((P, CW), dtype=np.uint8)
    wire = np.zeros(P, dtype=np.int64)
    for t in range(P):
        ref[t], wire[t] = enc.onTransmit(payload[t], int(lens[t]), t)
    got = closed_form_encode(oracle.gen_G(T, B, N), payload, lens, k, n, S, 300)
    assert (got == ref).all()
    nz = [np.flatnonzero(row) for row in ref]
    assert all(wire[t] == (nz[t][-1] + 1 if nz[t].size else 0) for t in range(P))


def test_encode_digests(oracle_vectors):
    for key, v in oracle_vectors["encode"].items():
        T, B, N = map(int, key.split(","))
        e = oracle.encode_stream(300, T, B, N, 0, v["packets"], seed=oracle_vectors["payload_seed"])
        assert hashlib.sha256(e["cw"].tobytes()).hexdigest() == v["codeword_sha256"]
        assert hashlib.sha256(e["cw_len"].astype("<i4").tobytes()).hexdigest() == v["wire_len_sha256"]


def test_decoder_created_midstream_and_startup_erasures():
    """Erasures inside the first T packets exercise the NULL-slot replay (Decoder.cpp:124-131)."""
    P = 400
    pat = np.zeros(P, dtype=np.uint8)
    pat[[0, 1, 3, 4, 5, 12, 13, 30, 31, 32, 33, 34, 35, 36]] = 1
    for tbn in [(10, 3, 3), (10, 5, 2), (10, 10, 10)]:
        r = oracle.run_stream(300, *tbn, P, pat, want_data=True)
        src = oracle.fill_payload(0, P, 300, 0x5EED)
        ok = r["out_len"] > 0
        assert (r["out_data"][ok] == src[ok]).all()
