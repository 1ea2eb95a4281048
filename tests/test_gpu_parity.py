"""Parity of the HIP path (through the C ABI) against the oracle.  Needs an MI355X: -m gpu.

Bit-exact comparisons at sizes the oracle finishes in seconds, plus size-independent properties
at BASELINE.json's full size (1M packets): encode -> erase -> decode round trip, lost set equal to
the (oracle-validated) symbolic planner's, payload lengths.
"""
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from conftest import ROOT, load_pattern

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import fec_erasure_code_unit_test_relay_amd as fec  # noqa: E402

L = 300
SEED = 0x5EED


@pytest.fixture(scope="module", autouse=True)
def device():
    assert torch.cuda.is_available(), "no HIP device"
    torch.cuda.set_device(0)
    yield


def test_fill_payload_matches_oracle_generator():
    g = fec.fill_payload(100, 50, L, SEED).cpu().numpy()
    assert (g == oracle.fill_payload(100, 50, L, SEED)).all()


ENC_CONFIGS = [(10, 3, 3), (10, 5, 2), (10, 1, 1), (10, 0, 0), (10, 2, 2), (10, 5, 5),
               (10, 7, 7), (10, 9, 9), (10, 10, 10), (10, 8, 4), (10, 5, 4), (10, 9, 8), (10, 4, 1),
               (4, 6, 2), (12, 4, 2), (10, 9, 1), (10, 10, 1)]


@pytest.mark.parametrize("path", ["generic", "auto", "tile"])
@pytest.mark.parametrize("tbn", ENC_CONFIGS)
def test_encode_bit_exact(tbn, path):
    T, B, N = tbn
    P = 2500
    c = fec.Codec(L, T, B, N)
    try:
        c.set_encode_path(path)
    except fec.FecError:
        pytest.skip(f"no {path} kernel for {tbn}")
    payload = fec.fill_payload(0, P, L, SEED)
    cw, wl = c.encode(payload)
    ref = oracle.encode_stream(L, T, B, N, 0, P, seed=SEED)
    assert (cw.cpu().numpy() == ref["cw"]).all()
    assert (wl.cpu().numpy() == ref["cw_len"]).all()
    assert (c.generator() == oracle.gen_G(T, B, N)).all()


def test_encode_other_payload_sizes():
    """Both encoders with payload sizes other than 300 (L % 4 == 0) and tiny batches."""
    for Lx, tbn, P in [(4, (10, 3, 3), 200), (64, (10, 5, 2), 300), (1500, (10, 3, 3), 130),
                       (300, (10, 3, 3), 1), (300, (10, 1, 1), 7), (1500, (10, 5, 2), 700)]:
        ref = oracle.encode_stream(Lx, *tbn, 0, P, seed=11)
        for path in ("generic", "tile"):
            c = fec.Codec(Lx, *tbn)
            try:
                c.set_encode_path(path)
            except fec.FecError:
                # tile: its LDS tile must hold the rows and the n-1 packets of parity history
                assert path == "tile" and Lx > 300
                continue
            payload = fec.fill_payload(0, P, Lx, 11)
            cw, wl = c.encode(payload)
            assert (cw.cpu().numpy() == ref["cw"]).all(), (Lx, tbn, path)
            assert (wl.cpu().numpy() == ref["cw_len"]).all(), (Lx, tbn, path)


@pytest.mark.parametrize("tbn", [(10, 3, 3), (10, 5, 2), (10, 1, 1), (10, 10, 10), (10, 0, 0)])
def test_encode_many_tiles_per_workgroup(tbn):
    """The tile kernel carries parity rows from tile to tile inside a workgroup: compare it with
    the generic kernel (itself checked against the oracle above) on a batch long enough for tens of
    tiles per workgroup, with random lengths and a history window."""
    P = 300_000
    rng = np.random.default_rng(17)
    lens = torch.from_numpy(rng.integers(0, L + 1, size=P).astype(np.int32)).cuda()
    payload = fec.fill_payload(0, P, L, 23)
    outs = []
    for path in ("generic", "tile"):
        c = fec.Codec(L, *tbn)
        try:
            c.set_encode_path(path)
        except fec.FecError:
            continue
        cw, wl = c.encode(payload, lens)
        h = 64  # second half with a history window (row offsets stay 16-byte aligned)
        cw2, wl2 = c.encode(payload[P // 2 - h:], lens[P // 2 - h:], history=h)
        outs.append((cw, wl, cw2, wl2))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)
        assert torch.equal(o[2], o[0][P // 2:])


@pytest.mark.parametrize("path", ["tile", "generic"])
@pytest.mark.parametrize("tbn", [(10, 3, 3), (10, 5, 2), (10, 1, 1), (10, 0, 0), (10, 9, 9)])
def test_encode_batch_edges(tbn, path):
    """The tile kernel splits a batch into workgroup runs of tiles with the tile in front: sizes
    around the tile length, odd batch ends (the last codeword's final partial dword) and both
    codeword alignments, against the oracle."""
    for P in (1, 2, 3, 5, 23, 24, 25, 41, 64, 1001, 4099, 70001):
        ref = oracle.encode_stream(L, *tbn, 0, P, seed=5)
        c = fec.Codec(L, *tbn)
        try:
            c.set_encode_path(path)
        except fec.FecError:
            pytest.skip(f"no {path} kernel for {tbn}")
        payload = fec.fill_payload(0, P, L, 5)
        cw, wl = c.encode(payload)
        assert (cw.cpu().numpy() == ref["cw"]).all(), (tbn, P)
        assert (wl.cpu().numpy() == ref["cw_len"]).all(), (tbn, P)


def test_encode_digest_fixture(oracle_vectors):
    for key, v in oracle_vectors["encode"].items():
        T, B, N = map(int, key.split(","))
        c = fec.Codec(L, T, B, N)
        cw, wl = c.encode(fec.fill_payload(0, v["packets"], L, SEED))
        assert hashlib.sha256(cw.cpu().numpy().tobytes()).hexdigest() == v["codeword_sha256"]
        assert hashlib.sha256(wl.cpu().numpy().astype("<i4").tobytes()).hexdigest() == v["wire_len_sha256"]


@pytest.mark.parametrize("path", ["generic", "tile"])
@pytest.mark.parametrize("tbn", [(10, 3, 3), (10, 5, 2), (10, 10, 10), (10, 9, 9), (10, 0, 0)])
def test_encode_variable_lengths_and_history(tbn, path):
    T, B, N = tbn
    P = 700
    rng = np.random.default_rng(3)
    lens = rng.integers(0, L + 1, size=P).astype(np.int32)
    lens[::7] = 0
    lens[1::11] = 1
    payload = fec.fill_payload(0, P, L, 9)
    enc = oracle.Encoder(L, T, B, N)
    host = payload.cpu().numpy()
    ref = np.stack([enc.onTransmit(host[t], int(lens[t]), t)[0] for t in range(P)])
    c = fec.Codec(L, T, B, N)
    try:
        c.set_encode_path(path)
    except fec.FecError:
        pytest.skip(f"no {path} kernel for {tbn}")
    dl = torch.from_numpy(lens).cuda()
    cw, _ = c.encode(payload, dl)
    assert (cw.cpu().numpy() == ref).all()
    # the same stream in two batches: the second sees 36 packets of history
    h, cut = 36, 400
    cw1, _ = c.encode(payload[:cut], dl[:cut])
    cw2, _ = c.encode(payload[cut - h:], dl[cut - h:], history=h)
    assert (torch.cat([cw1, cw2]).cpu().numpy() == ref).all()


def gpu_round_trip(T, B, N, pattern, P, garbage=True, path="auto", dedup=True):
    """GPU encode of packets 0..P+T-1, erase, GPU decode -> outputs for packets 0..P-1.
    path: kernel selection of the decoder's copy and planner ('auto', 'generic' or 'fast');
    dedup: planner replays one episode per loss shape (True) or every episode."""
    c = fec.Codec(L, T, B, N)
    try:
        c.set_copy_path(path)
        c.set_plan_path(path if path in ("generic", "auto") else "auto")
    except fec.FecError:
        pytest.skip(f"no {path} kernel for {(T, B, N)}")
    c.set_episode_dedup(dedup)
    Pf = P + T
    pat = np.zeros(Pf, dtype=np.uint8)
    m = min(pattern.size, Pf)
    pat[:m] = pattern[:m]
    payload = fec.fill_payload(0, Pf, L, SEED)
    cw, _ = c.encode(payload)
    er = torch.from_numpy(pat).cuda()
    if garbage:  # the decoder must never read an erased packet's bytes
        idx = torch.nonzero(er).flatten()
        if idx.numel():
            cw[idx] = torch.randint(0, 256, (idx.numel(), c.CW), dtype=torch.uint8, device="cuda")
    out, ln = c.decode(cw, er)
    torch.cuda.synchronize()
    return c, payload, out, ln, pat


DEC_CASES = [((10, 5, 2), "bin_erasure", 0, 8000), ((10, 3, 3), "bin_erasure", 0, 8000),
             ((10, 9, 8), "erasure100", 0, 4000), ((10, 1, 1), "erasure10", 50000, 6000),
             ((10, 4, 3), "erasure80", 10000, 6000), ((10, 10, 10), "erasure90", 0, 3000),
             ((10, 0, 0), "erasure70", 0, 5000), ((10, 8, 4), "erasure60", 0, 5000),
             ((12, 4, 2), "erasure100", 1000, 3000), ((4, 6, 2), "erasure100", 0, 3000),
             ((15, 2, 1), "erasure100", 0, 2000), ((16, 1, 1), "erasure90", 500, 2000),
             ((10, 4, 4), "bin_erasure", 2000, 6000), ((10, 5, 5), "erasure80", 0, 4000),
             # n = 18..21: no rule table, the planner's wave computes gf256_rref_matrix itself
             ((10, 9, 1), "erasure100", 0, 6000), ((10, 10, 1), "erasure100", 0, 6000),
             ((10, 8, 1), "erasure90", 2000, 5000), ((10, 9, 2), "erasure100", 7000, 5000)]


@pytest.mark.parametrize("path,dedup", [("generic", False), ("fast", True), ("auto", False), ("auto", True)])
@pytest.mark.parametrize("tbn,pattern,start,P", DEC_CASES)
def test_decode_bit_exact_vs_oracle(tbn, pattern, start, P, path, dedup):
    T, B, N = tbn
    pat = load_pattern(pattern)[start:start + P + T]
    ref = oracle.run_stream(L, T, B, N, P, pat, seed=SEED, want_data=True)
    c, payload, out, ln, _ = gpu_round_trip(T, B, N, pat, P, path=path, dedup=dedup)
    assert (ln.cpu().numpy() == ref["out_len"]).all()
    assert (out.cpu().numpy() == ref["out_data"]).all()
    eps, rec, lost = c.counters()
    assert lost == int((ref["out_len"] == 0).sum())  # every lost packet is an erased one
    assert rec + lost == int(pat[:P].sum())


def test_copy_fast_variable_lengths_and_sizes():
    """Received packets of every length (and other payload sizes) through the specialised copy."""
    for Lx, tbn in [(300, (10, 3, 3)), (300, (10, 10, 10)), (64, (10, 5, 2)), (1500, (10, 3, 3))]:
        T, B, N = tbn
        P = 700
        rng = np.random.default_rng(Lx)
        lens = rng.integers(0, Lx + 1, size=P + T).astype(np.int32)
        lens[::9] = Lx
        pat = (rng.random(P + T) < 0.05).astype(np.uint8)
        enc = oracle.Encoder(Lx, T, B, N)
        dec = oracle.Decoder(Lx, T, B, N)
        src = oracle.fill_payload(0, P + T, Lx, 5)
        cws, want_len, want = [], [], []
        for t in range(P + T):
            cw, size = enc.onTransmit(src[t], int(lens[t]), t)
            cws.append(cw)
            out, p = dec.onReceive(None if pat[t] else cw, size, t, bool(pat[t]))
            if t >= T:
                want.append(out)
                want_len.append(p)
        for cpath in ("fast", "generic"):
            c = fec.Codec(Lx, T, B, N)
            c.set_copy_path(cpath)
            out, ln = c.decode(torch.from_numpy(np.stack(cws)).cuda(), torch.from_numpy(pat).cuda())
            assert (ln.cpu().numpy() == np.array(want_len)).all(), (Lx, tbn, cpath)
            assert (out.cpu().numpy() == np.stack(want)).all(), (Lx, tbn, cpath)


def test_decode_startup_and_dense_erasures():
    P = 600
    pat = np.zeros(P + 10, dtype=np.uint8)
    pat[[0, 1, 3, 4, 5, 12, 13]] = 1
    pat[30:37] = 1
    pat[100:140:2] = 1
    pat[300:330] = 1
    for tbn in [(10, 3, 3), (10, 5, 2), (10, 10, 10), (10, 2, 2)]:
        ref = oracle.run_stream(L, *tbn, P, pat, seed=SEED, want_data=True)
        _, _, out, ln, _ = gpu_round_trip(*tbn, pat, P)
        assert (ln.cpu().numpy() == ref["out_len"]).all()
        assert (out.cpu().numpy() == ref["out_data"]).all()


def test_full_size_round_trip_1M():
    """BASELINE config 2/3 size: 1M packets at (10,3,3) with bin/erasure.bin tiled."""
    T, B, N = 10, 3, 3
    P = 1_000_000
    base = load_pattern("bin_erasure")[:360000]
    pat = np.resize(base, P + T).astype(np.uint8)
    c, payload, out, ln, _ = gpu_round_trip(T, B, N, pat, P, garbage=False)
    fate = fec.plan_host(L, T, B, N, pat)
    lost = fate == 3
    lnh = ln.cpu().numpy()
    assert ((lnh == 0) == lost).all()
    assert (lnh[~lost] == L).all()
    ok = torch.from_numpy(~lost).cuda()
    assert torch.equal(out[ok], payload[:P][ok])
    assert int(out[~ok].count_nonzero()) == 0
    eps, rec, nlost = c.counters()
    assert nlost == int(lost.sum()) and rec == int((fate == 2).sum())
    replayed, filled = c.plan_stats()
    assert replayed + filled == eps and filled > 0


def _check_recovered_equal_source(payload, out, ln, P):
    lnh = ln.cpu().numpy()
    ok = torch.from_numpy(lnh != 0).cuda()
    assert (lnh[lnh != 0] == L).all()
    assert torch.equal(out[ok], payload[:P][ok])
    return np.flatnonzero(lnh == 0)


def test_gpu_decode_reproduces_published_loss_counts(published_runs):
    """The reference's own published results (Experimental_Logs/Logs/Fixed/*Receiver*.rtf: `Final FEC
    loss rate` x 360000 on the shipped pattern) reproduced by the HIP decoder itself:
    12 (T,B,N, pattern) runs, 360 000 packets each, lost count exact, every other packet recovered
    byte for byte."""
    P = 360000
    for run in published_runs:
        T, B, N = run["T"], run["B"], run["N"]
        pat = load_pattern(run["pattern"])[:P]
        c, payload, out, ln, _ = gpu_round_trip(T, B, N, pat, P)
        lost = _check_recovered_equal_source(payload, out, ln, P)
        assert lost.size == run["lost_packets"], run["log"]


def test_gpu_lost_sets_equal_oracle_recorded_lists(oracle_vectors):
    """BASELINE config 3 (10,5,2) and (10,3,3) on bin/erasure.bin, 360 000 packets: the GPU's lost
    packets are exactly the oracle's recorded index lists (565 and 4662 packets)."""
    P = 360000
    pat = load_pattern("bin_erasure")[:P]
    for key, want in oracle_vectors["lost"].items():
        T, B, N = map(int, key.split(","))
        c, payload, out, ln, _ = gpu_round_trip(T, B, N, pat, P)
        lost = _check_recovered_equal_source(payload, out, ln, P)
        assert lost.tolist() == want, key


def test_episode_dedup_many_shapes():
    """Dense random losses (thousands of distinct shapes, long and truncated episodes) with and
    without deduplication: identical outputs, and equal to the host planner's fates."""
    T, B, N = 10, 3, 3
    P = 200_000
    rng = np.random.default_rng(7)
    pat = np.zeros(P + T, dtype=np.uint8)
    for s in rng.integers(0, P + T, size=6000):  # bursts of random length and density
        ln = int(rng.integers(1, 90))
        pat[s:s + ln] |= (rng.random(min(ln, P + T - s)) < rng.uniform(0.2, 1.0)).astype(np.uint8)
    pat[-5:] = 1  # an episode running into the batch end
    res = []
    for dedup in (False, True):
        c, payload, out, ln, _ = gpu_round_trip(T, B, N, pat, P, garbage=False, dedup=dedup)
        res.append((out.cpu().numpy(), ln.cpu().numpy(), c.counters(), c.plan_stats()))
    assert (res[0][0] == res[1][0]).all() and (res[0][1] == res[1][1]).all()
    assert res[0][2] == res[1][2]
    assert res[0][3][1] == 0 and res[1][3][1] > 0
    fate = fec.plan_host(L, T, B, N, pat)
    assert ((res[1][1] == 0) == (fate == 3)).all()


def test_streaming_api_matches_oracle():
    T, B, N = 10, 5, 2
    P = 500
    pat = load_pattern("bin_erasure")[2600:2600 + P + T].copy()
    pat[[3, 4, 200, 201, 202, 203]] = 1
    enc, dec = fec.FEC_Encoder(L, T, B, N), fec.FEC_Decoder(L, T, B, N)
    oe, od = oracle.Encoder(L, T, B, N), oracle.Decoder(L, T, B, N)
    src = oracle.fill_payload(0, P + T, L, SEED)
    lens = np.full(P + T, L)
    lens[50:60] = [0, 1, 2, 7, 100, 299, 300, 5, 33, 250]
    for t in range(P + T):
        wire, size = enc.onTransmit(src[t], int(lens[t]), t)
        ocw, osize = oe.onTransmit(src[t], int(lens[t]), t)
        assert size == osize and (wire == ocw[:size]).all()
        erased = bool(pat[t])
        got, p = dec.onReceive(None if erased else wire, size, t, erased)
        ogot, op = od.onReceive(None if erased else ocw, osize, t, erased)
        assert p == op and (got == ogot).all(), t


def test_streaming_api_across_server_idle_exits():
    """The per-packet coders' resident servers exit after 50 ms without a request (state back to
    HBM) and are relaunched by the next call (fec_server.hip, exit handshake): calls separated by
    pauses longer than that give the oracle's outputs, recovered packets included."""
    import time
    T, B, N = 10, 3, 3
    P = 120
    pat = np.zeros(P + T, dtype=np.uint8)
    pat[[20, 21, 22, 60, 61, 90]] = 1
    enc, dec = fec.FEC_Encoder(L, T, B, N), fec.FEC_Decoder(L, T, B, N)
    oe, od = oracle.Encoder(L, T, B, N), oracle.Decoder(L, T, B, N)
    src = oracle.fill_payload(0, P + T, L, SEED)
    for t in range(P + T):
        if t in (5, 31, 70, 100):
            time.sleep(0.12)
        wire, size = enc.onTransmit(src[t], L, t)
        ocw, osize = oe.onTransmit(src[t], L, t)
        assert size == osize and (wire == ocw[:size]).all(), t
        erased = bool(pat[t])
        got, p = dec.onReceive(None if erased else wire, size, t, erased)
        ogot, op = od.onReceive(None if erased else ocw, osize, t, erased)
        assert p == op and (got == ogot).all(), t


def test_streaming_api_many_coders_interleaved():
    """Six encoder/decoder pairs used in turn (12 coders, more than the process's persistent-server
    slots, FEC_SERVER_MAX = 1, and more streams than hardware queues): every call equals the oracle,
    recovered packets included, and no call waits out another coder's server (50 ms idle limit)."""
    import time
    T, B, N = 10, 3, 3
    P = 150
    pairs = []
    for c in range(6):
        pat = np.zeros(P + T, dtype=np.uint8)
        pat[[10 + c, 11 + c, 12 + c, 60, 61 + c, 100 + 2 * c]] = 1
        pairs.append((fec.FEC_Encoder(L, T, B, N), fec.FEC_Decoder(L, T, B, N),
                      oracle.Encoder(L, T, B, N), oracle.Decoder(L, T, B, N), pat))
    src = oracle.fill_payload(0, P + T, L, SEED)
    worst = 0.0
    for t in range(P + T):
        for enc, dec, oe, od, pat in pairs:
            t0 = time.perf_counter()
            wire, size = enc.onTransmit(src[t], L, t)
            erased = bool(pat[t])
            got, p = dec.onReceive(None if erased else wire, size, t, erased)
            worst = max(worst, time.perf_counter() - t0)
            ocw, osize = oe.onTransmit(src[t], L, t)
            ogot, op = od.onReceive(None if erased else ocw, osize, t, erased)
            assert size == osize and (wire == ocw[:size]).all(), t
            assert p == op and (got == ogot).all(), t
    assert worst < 0.025, f"a call took {worst * 1e3:.1f} ms"


def test_live_server_holds_no_other_launch():
    """A live per-packet server (FEC_Encoder's resident workgroup, polling for 50 ms after its last
    call) must not hold work launched elsewhere in the process behind it: with the encoder's server
    alive, torch kernels on six other streams and on the default stream, and a batched decode
    (fec_decode_batch on torch's current stream), each finish within 5 ms of their launch.  The
    coders' streams have the greatest priority, on hardware queues apart from normal streams
    (fec_codec.hip coder_stream_create); the encoder's calls stay equal to the oracle."""
    import time
    torch = pytest.importorskip("torch")
    T, B, N = 10, 3, 3
    torch.cuda.set_device(0)
    enc, oe = fec.FEC_Encoder(L, T, B, N), oracle.Encoder(L, T, B, N)
    src = oracle.fill_payload(0, 400, L, SEED)
    codec = fec.Codec(L, T, B, N)
    Pb = 20000
    cw, _ = codec.encode(fec.fill_payload(0, Pb, L, SEED))
    er = torch.from_numpy(load_pattern("bin_erasure")[:Pb].copy()).cuda()
    codec.workspace(Pb)
    streams = [torch.cuda.Stream() for _ in range(6)]
    xs = [torch.zeros(1 << 16, device="cuda") for _ in range(7)]
    for i, st in enumerate(streams):  # first use of each stream (queue set-up) before the server starts
        with torch.cuda.stream(st):
            xs[i].add_(0.0)
    codec.decode(cw, er)
    torch.cuda.synchronize()
    worst = {"stream": 0.0, "default": 0.0, "decode": 0.0}
    for t in range(40):
        wire, size = enc.onTransmit(src[t], L, t)  # the server is alive (50 ms idle limit)
        ocw, osize = oe.onTransmit(src[t], L, t)
        assert size == osize and (wire == ocw[:size]).all(), t
        for i, st in enumerate(streams):
            t0 = time.perf_counter()
            with torch.cuda.stream(st):
                xs[i].add_(1.0)
            st.synchronize()
            worst["stream"] = max(worst["stream"], time.perf_counter() - t0)
        t0 = time.perf_counter()
        xs[6].add_(1.0)  # default stream
        torch.cuda.current_stream().synchronize()
        worst["default"] = max(worst["default"], time.perf_counter() - t0)
        t0 = time.perf_counter()
        out, ln = codec.decode(cw, er)
        torch.cuda.current_stream().synchronize()
        worst["decode"] = max(worst["decode"], time.perf_counter() - t0)
    for i in range(7):
        assert float(xs[i][0]) == 40.0
    assert max(worst.values()) < 0.005, {k: round(v * 1e3, 2) for k, v in worst.items()}


def _bench_json(args, env):
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_config5_bench_two_ranks_gloo():
    """BASELINE config 5's partition at its per-GPU size (one independent stream of 1M packets per
    rank, no data-path collective): bench.py --gpus 2 starts two rank processes itself; on a one-GPU
    box they share the card and rendezvous over gloo (FEC_BENCH_BACKEND=gloo).  Both ranks verify
    their round trip, rank 0 reports the whole job, and each rank's counters and output digest equal
    a single-rank run of the same stream (--stream-id: the same payload seed and pattern phase)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR")}
    env["FEC_BENCH_BACKEND"] = "gloo"
    common = ["--steps", "3", "--warmup", "1", "--warm-seconds", "0.2", "--packets", "1000000",
              "--no-extra-configs", "--no-cpu-baseline", "--no-host-inclusive"]
    d = _bench_json(["--gpus", "2"] + common, env)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["verified"] is True  # every rank's round trip (bench.py reduces the flags over the ranks)
    assert d["config"]["packets_per_gpu"] == 1000000
    dec = d["decode"]  # summed over the two ranks
    assert dec["erased"] > 0 and dec["recovered"] + dec["lost"] == dec["erased"]
    ranks = d["per_rank"]
    assert [x["stream"] for x in ranks] == [0, 1]
    assert sum(x["erased"] for x in ranks) == dec["erased"] and sum(x["lost"] for x in ranks) == dec["lost"]
    assert ranks[0]["erased"] != ranks[1]["erased"]  # different phases of the pattern
    for sid in (0, 1):
        single = _bench_json(["--gpus", "1", "--stream-id", str(sid)] + common, env)
        assert single["per_rank"] == [ranks[sid]], (single["per_rank"], ranks[sid])


def test_cpp_dropin_program(tmp_path):
    """The reference-named C++ classes (include/fec_amd_dropin.h) in a host program."""
    src = os.path.join(ROOT, "tests", "cpp", "dropin_test.cpp")
    exe = str(tmp_path / "dropin_test")
    libdir = os.path.dirname(fec.LIB_PATH)
    orc = os.path.join(ROOT, "oracle", "fec_oracle.c")
    subprocess.run(["gcc", "-O2", "-c", orc, "-o", str(tmp_path / "oracle.o")], check=True)
    subprocess.run(["g++", "-O2", "-std=c++17", src, str(tmp_path / "oracle.o"), "-I",
                    os.path.join(ROOT, "include"), "-L", libdir, "-lfec_amd",
                    f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "DROPIN OK" in r.stdout


def test_plan_apply_split_on_two_streams_equals_decode():
    T, B, N = 10, 5, 2
    P = 20000
    pat = np.resize(load_pattern("bin_erasure")[:360000], P + T).astype(np.uint8)
    c, payload, out, ln, _ = gpu_round_trip(T, B, N, pat, P, garbage=False)
    cw, _ = c.encode(payload)
    er = torch.from_numpy(pat).cuda()
    side = torch.cuda.Stream()
    fork = torch.cuda.Event()
    fork.record()
    with torch.cuda.stream(side):
        side.wait_event(fork)
        c.plan(er)
    torch.cuda.current_stream().wait_stream(side)
    out2, ln2 = c.apply(cw, er)
    torch.cuda.synchronize()
    assert torch.equal(out, out2) and torch.equal(ln, ln2)


def _config_vectors():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "config_vectors.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("eps", ["0.0001", "0.01"])
def test_config1_iid_361000_bit_exact(eps):
    """BASELINE config 1: (10,3,3), 361 000 packets, i.i.d. erasures generate_IID(361010, eps,
    seed 0) (Erasure_File_Generator.cpp:25-63, the driver's EPSILON = 1e-4 and the heavier 1e-2).
    The HIP encode -> erase -> decode output (lengths and bytes) equals the oracle's, recorded in
    tests/golden/config_vectors.json."""
    from fec_erasure_code_unit_test_relay_amd.erasure import Erasure_File_Generator
    v = _config_vectors()["config1"][eps]
    P = v["packets"]
    pat = Erasure_File_Generator().generate_IID(P + 10, float(eps), seed=0)
    assert hashlib.sha256(pat.tobytes()).hexdigest() == v["pattern_sha256"]
    assert np.flatnonzero(pat).tolist() == v["erased"]
    c, payload, out, ln, _ = gpu_round_trip(10, 3, 3, pat, P)
    lnh = ln.cpu().numpy()
    assert np.flatnonzero(lnh == 0).tolist() == v["lost"]
    assert hashlib.sha256(lnh.astype("<i4").tobytes()).hexdigest() == v["out_len_sha256"]
    assert hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == v["out_data_sha256"]


def test_config2_full_size_digest():
    """BASELINE config 2: 1 000 010 packets (the bench's encoded batch) at (10,3,3): SHA-256 of the
    codewords and wire sizes equal the oracle's (tests/golden/config_vectors.json)."""
    v = _config_vectors()["config2"]
    c = fec.Codec(L, v["T"], v["B"], v["N"])
    cw, wl = c.encode(fec.fill_payload(0, v["packets"], L, SEED))
    assert hashlib.sha256(cw.cpu().numpy().tobytes()).hexdigest() == v["codeword_sha256"]
    assert hashlib.sha256(wl.cpu().numpy().astype("<i4").tobytes()).hexdigest() == v["wire_len_sha256"]


def test_encode_chunked_batch_with_long_history():
    """A batch beyond the wave kernel's 32-bit addressing (> 2 GB of codewords) is encoded in
    chunks; a history longer than n-1 rows must not change that (it used to recurse forever)."""
    T, B, N = 10, 3, 3
    h, P = 36, 5_400_000
    c = fec.Codec(L, T, B, N)
    payload = fec.fill_payload(0, P + h, L, 31)
    a, al = c.encode(payload[h:])                 # encoder created at row h
    b, bl = c.encode(payload, history=h)          # the same rows after h rows of history
    full, fl = c.encode(payload[h - (c.n - 1):], history=c.n - 1)
    assert torch.equal(b, full) and torch.equal(bl, fl)
    # rows >= n-1 of the history-less batch see the same n-1 packets in front
    assert torch.equal(a[c.n - 1:], b[c.n - 1:])
    del a, b, full


@pytest.mark.parametrize("tbn,start", [((10, 3, 3), 1234), ((10, 5, 2), 77777), ((10, 10, 10), 5)])
def test_streaming_api_starts_mid_stream(tbn, start):
    """Variable_Rate_FEC_Encoder/Decoder construct coders mid-stream and call them with the global
    sequence number (Variable_Rate_FEC_Encoder.cpp:126/144/185, Variable_Rate_FEC_Decoder.cpp:2472/
    2524): the first seq is the coder's origin.  Against the oracle (which, like the reference,
    indexes by seq % n from an all-zero state) fed the same absolute seqs."""
    T, B, N = tbn
    P = 300
    pat = load_pattern("bin_erasure")[3300:3300 + P + T].copy()
    pat[[0, 2, 150, 151, 152]] = 1
    enc, dec = fec.FEC_Encoder(L, T, B, N), fec.FEC_Decoder(L, T, B, N)
    oe, od = oracle.Encoder(L, T, B, N), oracle.Decoder(L, T, B, N)
    src = oracle.fill_payload(start, P + T, L, SEED)
    for i in range(P + T):
        t = start + i
        wire, size = enc.onTransmit(src[i], L, t)
        ocw, osize = oe.onTransmit(src[i], L, t)
        assert size == osize and (wire == ocw[:size]).all(), t
        erased = bool(pat[i])
        got, p = dec.onReceive(None if erased else wire, size, t, erased)
        ogot, op = od.onReceive(None if erased else ocw, osize, t, erased)
        assert p == op and (got == ogot).all(), t
    with pytest.raises(fec.FecError):
        enc.onTransmit(src[0], L, start + P + T + 5)  # later calls stay consecutive


def _stream_in_batches(c, cw, er_dev, pat, cuts, history_cap=None):
    """Push packets [cuts[i], cuts[i+1]) one batch at a time; every push gets the whole stream in
    front of it as history (or at most history_cap packets).  Returns the concatenated outputs."""
    ds = fec.DecodeStream(c)
    outs, lens = [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        h = a if history_cap is None else min(a, history_cap)
        o, ln = ds.push(cw[a - h:b], er_dev[a - h:b], pat[a - h:b], history=h)
        outs.append(o.clone())
        lens.append(ln.clone())
    return torch.cat(outs), torch.cat(lens), ds


def test_continuing_decode_1M_in_uneven_batches_equals_one_shot():
    """One 1M-packet stream (bin/erasure.bin tiled, (10,3,3)) decoded in 7 uneven batches through
    fec_decode_stream_push (the decoder state carried across calls) equals the one-shot decode,
    row for row, with cuts that fall inside erasure episodes."""
    T, B, N = 10, 3, 3
    P = 1_000_000
    pat = np.resize(load_pattern("bin_erasure")[:360000], P + T).astype(np.uint8)
    c = fec.Codec(L, T, B, N)
    payload = fec.fill_payload(0, P + T, L, SEED)
    cw, _ = c.encode(payload)
    er = torch.from_numpy(pat).cuda()
    ref, ref_len = c.decode(cw, er)
    # batch ends on and next to erased packets (mid-episode restarts)
    ers = np.flatnonzero(pat[:P])
    cuts = [0, 1, 7, int(ers[100]) + 1, int(ers[2000]) + 3, 400_001, int(ers[9000]), P + T]
    out, ln, ds = _stream_in_batches(c, cw, er, pat, cuts)
    torch.cuda.synchronize()
    assert out.shape[0] == P
    assert torch.equal(ln, ref_len)
    assert torch.equal(out, ref)
    assert ds.state()[0] == P + T


@pytest.mark.parametrize("tbn,pattern", [((10, 3, 3), "erasure50"), ((10, 5, 2), "bin_erasure"),
                                         ((10, 1, 1), "erasure90")])
def test_continuing_decode_vs_oracle(tbn, pattern):
    """Continuing decode in batches of 1..997 packets, with only the last 300 packets kept as
    history, against the oracle's FEC_Decoder fed the same stream packet by packet."""
    T, B, N = tbn
    P = 12000
    pat = load_pattern(pattern)[:P + T].astype(np.uint8)
    c = fec.Codec(L, T, B, N)
    payload = fec.fill_payload(0, P + T, L, SEED)
    cw, _ = c.encode(payload)
    er = torch.from_numpy(pat).cuda()
    rng = np.random.default_rng(5)
    cuts = [0]
    while cuts[-1] < P + T:
        cuts.append(min(P + T, cuts[-1] + int(rng.choice([1, 2, 11, 64, 250, 997]))))
    try:
        out, ln, _ = _stream_in_batches(c, cw, er, pat, cuts, history_cap=300)
    except fec.FecError as e:  # an episode longer than the history kept: say so, keep more
        assert e.status == fec._lib.FEC_ERR_HISTORY
        out, ln, _ = _stream_in_batches(c, cw, er, pat, cuts)
    torch.cuda.synchronize()
    ref = oracle.run_stream(L, T, B, N, P, pat, seed=SEED, want_data=True)
    assert (ln.cpu().numpy() == ref["out_len"]).all()
    assert (out.cpu().numpy() == ref["out_data"]).all()


def test_continuing_decode_reports_short_history():
    """A push whose kept history holds no restart point (an erasure every few packets) fails with
    FEC_ERR_HISTORY instead of decoding from a wrong state."""
    T, B, N = 10, 3, 3
    P = 400
    pat = np.zeros(P + T, dtype=np.uint8)
    pat[::5] = 1
    c = fec.Codec(L, T, B, N)
    cw, _ = c.encode(fec.fill_payload(0, P + T, L, SEED))
    er = torch.from_numpy(pat).cuda()
    ds = fec.DecodeStream(c)
    ds.push(cw[:200], er[:200], pat[:200], history=0)
    with pytest.raises(fec.FecError) as e:
        ds.push(cw[200 - 20:P + T], er[200 - 20:P + T], pat[200 - 20:P + T], history=20)
    assert e.value.status == fec._lib.FEC_ERR_HISTORY


@pytest.mark.parametrize("tbn,pattern", [((10, 3, 3), "bin_erasure"), ((10, 5, 2), "erasure50"),
                                         ((10, 1, 1), "erasure90"), ((10, 0, 0), "erasure10")])
def test_stream_group_equals_per_stream_coders(tbn, pattern):
    """37 independent streams, each call carrying the next packet of a random subset of them (one
    launch per call): every stream's codewords and sizes equal a fresh FEC_Encoder's over that
    stream alone, and every stream's decoded rows equal the one-shot decoder's (the oracle-checked
    batch decode) over its own erasure pattern -- a different phase of the shipped pattern each."""
    T, B, N = tbn
    ns, P = 37, 600
    base = load_pattern(pattern).astype(np.uint8)
    pats = [base[(s * 7919) % (base.size - P - T):][:P + T] for s in range(ns)]
    payloads = [fec.fill_payload(0, P + T, L, SEED + s) for s in range(ns)]
    c = fec.Codec(L, T, B, N)
    ref_cw, ref_out = [], []
    for s in range(ns):
        cw, wl = c.encode(payloads[s])
        o, ol = c.decode(cw, torch.from_numpy(pats[s]).cuda())
        ref_cw.append((cw, wl))
        ref_out.append((o, ol))
    grp = fec.StreamGroup(L, T, B, N, ns)
    rng = np.random.default_rng(11)
    sent = np.zeros(ns, dtype=np.int64)
    got_cw = [[] for _ in range(ns)]
    got_out = [[] for _ in range(ns)]
    while (sent < P + T).any():
        live = np.flatnonzero(sent < P + T)
        ids = rng.permutation(live)[:max(1, int(rng.integers(1, live.size + 1)))].astype(np.int32)
        pay = torch.stack([payloads[s][sent[s]] for s in ids])
        cw, wl = grp.encode(ids, pay)
        er = np.array([pats[s][sent[s]] for s in ids], dtype=np.uint8)
        out, ol = grp.decode(ids, er, cw)
        torch.cuda.synchronize()
        for j, s in enumerate(ids):
            got_cw[s].append((cw[j].clone(), wl[j].clone()))
            got_out[s].append((out[j].clone(), ol[j].clone()))
        sent[ids] += 1
    for s in range(ns):
        cw = torch.stack([x[0] for x in got_cw[s]])
        wl = torch.stack([x[1] for x in got_cw[s]])
        assert torch.equal(cw, ref_cw[s][0]) and torch.equal(wl, ref_cw[s][1]), s
        out = torch.stack([x[0] for x in got_out[s]])[T:]
        ol = torch.stack([x[1] for x in got_out[s]])
        assert bool((ol[:T] == 0).all()), s
        assert torch.equal(ol[T:], ref_out[s][1]), s
        assert torch.equal(out, ref_out[s][0]), s


def test_stream_group_calls_on_alternating_streams():
    """Consecutive group calls on two different HIP streams, with no wait between them in the
    caller beyond its own data (a decode waits for the encode whose codewords it reads): the group's
    staging buffer, windows and rings are ordered by the library itself, so every packet equals the
    single-stream run's."""
    T, B, N = 10, 3, 3
    ns, P = 64, 120
    base = load_pattern("bin_erasure").astype(np.uint8)
    pats = np.stack([base[s * 131: s * 131 + P] for s in range(ns)])
    pays = fec.fill_payload(0, P * ns, L, SEED).view(P, ns, L)
    ids = np.arange(ns, dtype=np.int32)

    def run(streams):
        grp = fec.StreamGroup(L, T, B, N, ns)
        cws = torch.empty((P, ns, grp.CW), dtype=torch.uint8, device="cuda")
        wls = torch.empty((P, ns), dtype=torch.int32, device="cuda")
        outs = torch.zeros((P, ns, L), dtype=torch.uint8, device="cuda")
        ols = torch.zeros((P, ns), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        for r in range(P):
            se, sd = streams[r % len(streams)], streams[(r + 1) % len(streams)]
            with torch.cuda.stream(se):
                grp.encode(ids, pays[r], out=cws[r], out_len=wls[r])
                ev = torch.cuda.Event()
                ev.record()
            with torch.cuda.stream(sd):
                sd.wait_event(ev)  # the caller's own dependency: codewords of this round
                grp.decode(ids, pats[:, r], cws[r], out=outs[r], out_len=ols[r])
        torch.cuda.synchronize()
        return cws, wls, outs, ols

    ref = run([torch.cuda.current_stream()])
    got = run([torch.cuda.Stream(), torch.cuda.Stream()])
    for a, b in zip(ref, got):
        assert torch.equal(a, b)


def test_stream_group_rejects_repeated_ids():
    grp = fec.StreamGroup(L, 10, 3, 3, 8)
    pay = fec.fill_payload(0, 2, L, SEED)
    with pytest.raises(fec.FecError):
        grp.encode(np.array([3, 3], dtype=np.int32), pay)
