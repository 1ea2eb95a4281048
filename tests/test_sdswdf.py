"""Relay state-dependent symbol-wise decode-and-forward (SD-SWDF, RELAYING_TYPE 3).

Reference: Decoder_Symbol_Wise::symbol_wise_encode_state_dependent (Decoder_Symbol_Wise.cpp:178-432),
symbol_wise_decode_state_dependent (:487-546) + extract_data (:653-661), driven with one relay frame
per seq (Variable_Rate_FEC_Decoder.cpp:636-675, 1458-1493, 1703-1721, 1798-1815).

CPU: the oracle's reference-structured chain (oracle/fec_oracle.c or_sdswdf_*) delivers every source
packet through clean hops with delay n1+n2-k-1, its outputs do not depend on the stale temp_codeword
bytes the reference leaves in place, and the library's host planner (fec_sdswdf_relay_plan /
fec_sdswdf_dest_plan) applied to the bytes in numpy gives the oracle's frames, outputs and flags on
three of the reference's shipped erasure recordings.  GPU: the HIP relay and destination kernels
give the same bytes.  Parity is against the oracle restatement (the reference ships no relay output:
parity unpinned by reference data).
"""
import numpy as np
import pytest

import oracle
from conftest import load_pattern

L = 300
SEED = 0x5EED
HDR = 11

# (T1, N1, T2, N2): k = T1-N1+1 = T2-N2+1, T2 <= T1 <= T_TOT
SD_CASES = [(10, 3, 10, 3), (10, 3, 9, 2), (10, 5, 8, 3), (10, 1, 10, 1), (6, 2, 5, 1), (10, 4, 10, 4)]
# three shipped recordings (bin/erasure.bin, bin/erasure2.bin, Experimental_Logs/erasure70.bin) for hop 1
# and hop 2, windows that hold bursts
PATTERNS = [("bin_erasure", 3000, "bin_erasure2", 9000), ("bin_erasure2", 21000, "erasure70", 5000),
            ("erasure70", 12000, "bin_erasure", 30000)]

_MUL = None


def gf_mul_table():
    global _MUL
    if _MUL is None:
        exp = np.zeros(512, dtype=np.int64)
        log = np.zeros(256, dtype=np.int64)
        x = 1
        for i in range(255):
            exp[i] = x
            log[x] = i
            x <<= 1
            if x & 0x100:
                x ^= 0x11D
        exp[255:510] = exp[:255]
        a = np.arange(256)
        m = exp[(log[:, None] + log[None, :])].astype(np.uint8)
        m[0, :] = 0
        m[:, 0] = 0
        _MUL = m
    return _MUL


def geometry(T1, N1, T2, N2):
    k, n1, n2 = T1 - N1 + 1, T1 + 1, T2 + 1
    S = -(-(L + 2) // k)
    return k, n1, n2, S, L // k + 1, 2 + HDR + (S + 1) * n2


def apply_relay(cw, ids, rec, T1, N1, T2, N2):
    """The relay plan applied to the source codeword bytes (numpy, test side)."""
    k, n1, n2, S, blocks, F = geometry(T1, N1, T2, N2)
    M = gf_mul_table()
    P = ids.size
    r = rec[ids]
    coef = r[:, HDR:].reshape(P, n2, n1)
    size = (S + 1) * n2
    fr = np.zeros((P, F), dtype=np.uint8)
    fr[:, 0] = size >> 8
    fr[:, 1] = size & 255
    fr[:, 2:2 + HDR] = r[:, :HDR]
    t = np.arange(P)
    jj = np.arange(blocks)
    for index in range(n2):
        acc = np.zeros((P, blocks), dtype=np.uint8)
        for p in range(n1):
            u = t - (n1 - 1) + p + (k - 1 - index)
            c = coef[:, index, p]
            ok = (u >= 0) & (c != 0)
            v = cw[np.clip(u, 0, P - 1)[:, None], (jj * n1 + p)[None, :]]
            acc ^= np.where(ok[:, None], M[c[:, None], v], 0).astype(np.uint8)
        fr[:, 4 + HDR + jj * n2 + index] = acc
    return fr


def apply_dest(frames, ids, rec, T1, N1, T2, N2):
    k, n1, n2, S, blocks, F = geometry(T1, N1, T2, N2)
    M = gf_mul_table()
    P = ids.size
    coef = rec[ids].reshape(P, k, n2)
    out = np.zeros((P, S * k), dtype=np.uint8)
    t = np.arange(P)
    jj = np.arange(blocks)
    for s in range(k):
        acc = np.zeros((P, blocks), dtype=np.uint8)
        for q in range(n2):
            u = t - s - (n2 - 1 - q)
            c = coef[:, s, q]
            ok = (u >= 0) & (c != 0)
            v = frames[np.clip(u, 0, P - 1)[:, None], (4 + HDR + jj * n2 + q)[None, :]]
            acc ^= np.where(ok[:, None], M[c[:, None], v], 0).astype(np.uint8)
        out[:, jj * k + s] = acc
    return out


def patterns(i, P):
    a, oa, b, ob = PATTERNS[i]
    e1 = load_pattern(a)[oa:oa + P].copy()
    e2 = load_pattern(b)[ob:ob + P].copy()
    e1[[0, 1, 2, 3, 300, 301, 303, 305, 307]] = 1  # start-up and dense windows
    e2[[5, 6, 600, 602, 604, 606]] = 1
    return e1, e2


def source_dwh(P, S, k):
    src = oracle.fill_payload(0, P, L, SEED)
    d = np.zeros((P, S * k), dtype=np.uint8)
    d[:, 0] = L >> 8
    d[:, 1] = L & 255
    d[:, 2:2 + L] = src
    return d


@pytest.mark.parametrize("cfg", SD_CASES)
def test_oracle_sdswdf_clean_hops_deliver_every_packet(cfg):
    P = 120
    z = np.zeros(P, dtype=np.uint8)
    r = oracle.sdswdf_run(L, *cfg, P, z, z, seed=SEED)
    D, S, k = r["delay"], r["S"], r["k"]
    nb = (L // k + 1) * k  # the relayed blocks (ceil(max_payload/k)+1 on ints)
    want = source_dwh(P, S, k)
    assert (r["dest_out"][D:, :nb] == want[:P - D, :nb]).all()
    assert (r["dest_out"][:, nb:] == 0).all()
    assert r["dest_flag"].sum() == 0
    # every clean frame carries the systematic header 1..n2 (then the untouched rows' 1-based indices)
    assert (r["frames"][:, 2:2 + HDR] == np.arange(1, HDR + 1)).all()


def test_oracle_sdswdf_outputs_ignore_stale_temp_codeword():
    """The reference leaves bytes of the previous diagonal in temp_codeword where a partial diagonal
    does not fill it (Decoder_Symbol_Wise.cpp:248-250): they never reach a frame or an output."""
    P = 900
    e1, e2 = patterns(0, P)
    a = oracle.sdswdf_run(L, 10, 3, 10, 3, P, e1, e2, seed=SEED, garbage=0)
    b = oracle.sdswdf_run(L, 10, 3, 10, 3, P, e1, e2, seed=SEED, garbage=0xA5)
    for key in ("frames", "dest_out", "dest_flag"):
        assert (a[key] == b[key]).all(), key
    assert a["dest_flag"].sum() > 0  # the window holds undecodable diagonals
    assert ((a["frames"][:, 2:2 + HDR] != np.arange(1, HDR + 1)).any(axis=1)).sum() > 0  # headers moved


def test_oracle_sdswdf_sdbo_flag_changes_burst_frames():
    """FLAG_FOR_SDBO = 1 (FEC_Macro.h:50 ships 0) turns on the burst branch (:230-231, :262-265,
    :303-305): frames change only around bursts longer than N."""
    P = 400
    e1 = np.zeros(P, dtype=np.uint8)
    e2 = np.zeros(P, dtype=np.uint8)
    e1[100:105] = 1  # a burst of 5 > N = 3
    a = oracle.sdswdf_run(L, 10, 3, 10, 3, P, e1, e2, seed=SEED, sdbo=0)
    b = oracle.sdswdf_run(L, 10, 3, 10, 3, P, e1, e2, seed=SEED, sdbo=1)
    diff = np.nonzero((a["frames"] != b["frames"]).any(axis=1))[0]
    assert diff.size > 0 and diff.min() >= 100 and diff.max() < 130


@pytest.mark.parametrize("pi", range(len(PATTERNS)))
@pytest.mark.parametrize("cfg", SD_CASES[:4])
def test_host_plan_equals_oracle(cfg, pi):
    """The library's host planner, its records applied to the bytes in numpy, against the oracle's
    frames, destination outputs and destination flags per seq."""
    from fec_erasure_code_unit_test_relay_amd.relay import StateDependentRelay
    P = 700
    e1, e2 = patterns(pi, P)
    ref = oracle.sdswdf_run(L, *cfg, P, e1, e2, seed=SEED)
    T1, N1, T2, N2 = cfg
    cw = oracle.encode_stream(L, T1, N1, N1, 0, P, seed=SEED)["cw"].copy()
    rng = np.random.default_rng(7)
    cw[e1[:P] == 1] = rng.integers(0, 256, (int(e1[:P].sum()), cw.shape[1]), dtype=np.uint8)
    r = StateDependentRelay(L, *cfg)
    assert r.frame_bytes == ref["frames"].shape[1] and r.delay == ref["delay"]
    ids, rec = r.relay_plan(e1)
    frames = apply_relay(cw, ids, rec, *cfg)
    assert (frames == ref["frames"]).all()
    fr2 = frames.copy()
    fr2[e2[:P] == 1] = rng.integers(0, 256, (int(e2[:P].sum()), fr2.shape[1]), dtype=np.uint8)
    did, drec, dfl = r.dest_plan(e2, fr2[:, 2:2 + HDR])
    out = apply_dest(fr2, did, drec, *cfg)
    assert (dfl == ref["dest_flag"]).all()
    assert (out == ref["dest_out"]).all()
    assert rec.shape[0] < P // 4  # plans repeat: an erasure-free stretch is one record


def test_host_plan_long_run_equals_oracle():
    """20 000 packets of the shipped patterns: the planners' memo tables (open addressing, grown at
    half load) grow several times, and the destination's sliding state key crosses thousands of
    states; frames, outputs and flags against the oracle."""
    from fec_erasure_code_unit_test_relay_amd.relay import StateDependentRelay
    from conftest import load_pattern
    P = 20000
    e1 = np.ascontiguousarray(load_pattern("bin_erasure")[:P + 40]).astype(np.uint8)
    e2 = np.ascontiguousarray(load_pattern("bin_erasure2")[:P + 40]).astype(np.uint8)
    cfg = (10, 3, 10, 3)
    ref = oracle.sdswdf_run(L, *cfg, P, e1, e2, seed=SEED)
    cw = oracle.encode_stream(L, 10, 3, 3, 0, P, seed=SEED)["cw"]
    r = StateDependentRelay(L, *cfg)
    ids, rec = r.relay_plan(e1[:P])
    frames = apply_relay(cw, ids, rec, *cfg)
    assert (frames == ref["frames"]).all()
    did, drec, dfl = r.dest_plan(e2[:P], frames[:, 2:2 + HDR])
    assert (dfl == ref["dest_flag"]).all()
    assert (apply_dest(frames, did, drec, *cfg) == ref["dest_out"]).all()


def test_host_plan_sdbo_equals_oracle():
    from fec_erasure_code_unit_test_relay_amd.relay import StateDependentRelay
    P = 700
    e1, e2 = patterns(1, P)
    e1[200:206] = 1
    ref = oracle.sdswdf_run(L, 10, 3, 10, 3, P, e1, e2, seed=SEED, sdbo=1)
    cw = oracle.encode_stream(L, 10, 3, 3, 0, P, seed=SEED)["cw"]
    r = StateDependentRelay(L, 10, 3, 10, 3, sdbo=1)
    ids, rec = r.relay_plan(e1)
    frames = apply_relay(cw, ids, rec, 10, 3, 10, 3)
    assert (frames == ref["frames"]).all()
    did, drec, dfl = r.dest_plan(e2, frames[:, 2:2 + HDR])
    assert (apply_dest(frames, did, drec, 10, 3, 10, 3) == ref["dest_out"]).all()
    assert (dfl == ref["dest_flag"]).all()


def test_sdswdf_rejects_unsupported_configurations():
    from fec_erasure_code_unit_test_relay_amd import FecError
    from fec_erasure_code_unit_test_relay_amd.relay import StateDependentRelay
    # ... and n2 = 1 (T2 = N2 = 0 with T1 = N1: k = 1), whose frame cannot hold its blocks
    for cfg in [(10, 3, 9, 3), (10, 3, 11, 4), (11, 3, 11, 3), (8, 2, 10, 4), (3, 3, 0, 0)]:
        with pytest.raises(FecError):
            StateDependentRelay(L, *cfg)


def test_sd_tile_kernel_fallback_geometry():
    """CPU (host geometry only): which type-3 batches take the tile kernel.  A tile holds at most 64
    packets (the kernel's record-id slots in LDS); round 5's two-packets-per-lane build
    (FEC_SD_PASS=2) made k = 11 tiles of 72 packets at L = 300 that overran them, so a garbage
    record id faulted the GPU -- the HIP error of r05zp, reproduced with that build in r06g
    (DESIGN §5).  The fallback is chosen for any tile over 64 packets, e.g. k = 11 at a 40-byte
    payload (S = 4: one lane per packet, 256 packets per tile)."""
    import ctypes
    from fec_erasure_code_unit_test_relay_amd._lib import lib
    tp, lds = ctypes.c_int(), ctypes.c_int()
    for relay in (1, 0):
        for N in range(0, 8):  # config 4's codes at L = 300: (10, N) -> (10, N), k = 11 - N
            assert lib().fec_sdswdf_tile_geometry(relay, L, 10, N, 10, N, 0, ctypes.byref(tp), ctypes.byref(lds)) == 1
            assert 0 < tp.value <= 64 and lds.value <= 65536, (relay, N, tp.value, lds.value)
        assert lib().fec_sdswdf_tile_geometry(relay, 40, 10, 0, 10, 0, 0, ctypes.byref(tp), ctypes.byref(lds)) == 0
        assert tp.value == 0
        # no tile kernel instantiated for (k, n1, n2) = (1, 11, 11): the per-(packet, block) kernel
        assert lib().fec_sdswdf_tile_geometry(relay, L, 10, 10, 10, 10, 0, ctypes.byref(tp), ctypes.byref(lds)) == 0
    assert lib().fec_sdswdf_tile_geometry(1, L, 10, 3, 9, 3, 0, ctypes.byref(tp), ctypes.byref(lds)) < 0


@pytest.mark.gpu
@pytest.mark.parametrize("pi", range(len(PATTERNS)))
@pytest.mark.parametrize("cfg", SD_CASES)
def test_gpu_sdswdf_bit_exact_vs_oracle(cfg, pi):
    """HIP relay frames, destination data_with_header rows and flags per seq against the oracle, on
    three shipped recordings; erased rows and frames are filled with garbage (never read)."""
    torch = pytest.importorskip("torch")
    import fec_erasure_code_unit_test_relay_amd as fec
    from fec_erasure_code_unit_test_relay_amd.relay import StateDependentRelay
    T1, N1, T2, N2 = cfg
    P = 1500
    e1, e2 = patterns(pi, P)
    ref = oracle.sdswdf_run(L, *cfg, P, e1, e2, seed=SEED)
    torch.cuda.set_device(0)
    c = fec.Codec(L, T1, N1, N1)
    cw, _ = c.encode(fec.fill_payload(0, P, L, SEED))
    idx = torch.from_numpy(np.nonzero(e1)[0]).cuda()
    cw[idx] = torch.randint(0, 256, (idx.numel(), c.CW), dtype=torch.uint8, device="cuda")
    r = StateDependentRelay(L, *cfg)
    frames = r.relay(cw, e1)
    fr2 = frames.clone()
    idx2 = torch.from_numpy(np.nonzero(e2)[0]).cuda()
    fr2[idx2] = torch.randint(0, 256, (idx2.numel(), r.frame_bytes), dtype=torch.uint8, device="cuda")
    out, dflag = r.destination(fr2, e2)
    torch.cuda.synchronize()
    assert (frames.cpu().numpy() == ref["frames"]).all()
    assert (out.cpu().numpy() == ref["dest_out"]).all()
    assert (dflag == ref["dest_flag"]).all()


@pytest.mark.gpu
def test_gpu_sdswdf_large_batch_round_trip():
    """360 000 packets through relay and destination with bin/erasure.bin on hop 1 (an erasure the
    relay cannot decode is still forwarded symbol by symbol): every destination row whose flag is
    clear and whose source window was decodable equals its source packet; the clean-hop run
    delivers every packet (size-independent properties at BASELINE scale)."""
    torch = pytest.importorskip("torch")
    import fec_erasure_code_unit_test_relay_amd as fec
    from fec_erasure_code_unit_test_relay_amd.relay import StateDependentRelay
    P = 360_000
    torch.cuda.set_device(0)
    c = fec.Codec(L, 10, 3, 3)
    payload = fec.fill_payload(0, P, L, SEED)
    cw, _ = c.encode(payload)
    r = StateDependentRelay(L, 10, 3, 10, 3)
    z = np.zeros(P, dtype=np.uint8)
    frames = r.relay(cw, z)
    out, dflag = r.destination(frames, z)
    D = r.delay
    assert int(dflag.sum()) == 0
    assert torch.equal(out[D:, 2:2 + L], payload[:P - D])
    e1 = load_pattern("bin_erasure")[:P].copy()
    frames = r.relay(cw, e1)
    out, dflag = r.destination(frames, z)
    good = (out[D:, 2:2 + L] == payload[:P - D]).all(dim=1).cpu().numpy()
    assert good.mean() > 0.98


def _build_relay_driver(tmp_path, oracle_only):
    import os
    import shutil
    import subprocess
    from conftest import ROOT
    import fec_erasure_code_unit_test_relay_amd as fec
    if shutil.which("g++") is None or not os.path.exists(fec.LIB_PATH):
        pytest.skip("needs g++ and the built libfec_amd.so")
    libdir = os.path.dirname(fec.LIB_PATH)
    exe = str(tmp_path / ("relay_oracle" if oracle_only else "relay_dropin"))
    cmd = ["g++", "-O2", "-std=c++17", "-x", "c++", os.path.join(ROOT, "tests", "cpp", "relay_dropin_test.cpp"),
           "-x", "c", os.path.join(ROOT, "oracle", "fec_oracle.c"), "-x", "none",
           "-I", os.path.join(ROOT, "include"), "-L", libdir, "-lfec_amd", f"-Wl,-rpath,{libdir}", "-o", exe]
    if oracle_only:
        cmd.insert(1, "-DRELAY_ORACLE_ONLY")
    subprocess.run(cmd, check=True, timeout=300)
    return exe


def test_relay_driver_over_oracle_methods_equals_oracle_chains(tmp_path):
    """tests/cpp/relay_dropin_test.cpp drives the reference's Decoder_Symbol_Wise member arrays the
    way Variable_Rate_FEC_Decoder does (types 2 and 3); over the oracle's per-call methods (or_sw_*,
    the signatures of the product's fec_sw_* C ABI) it reproduces the oracle's whole relay chains."""
    import subprocess
    exe = _build_relay_driver(tmp_path, oracle_only=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "RELAY ORACLE DRIVER OK" in r.stdout


@pytest.mark.gpu
def test_gpu_relay_dropin_class_equals_oracle(tmp_path):
    """siphon::Decoder_Symbol_Wise (include/fec_amd_dropin.h, GF work through fec_sw_* on the GPU)
    under the same driver: frames, destination outputs and flags equal the oracle's chains at fixed
    rate, and equal the oracle-method class through a double-coding transition (copy_elements)."""
    import subprocess
    exe = _build_relay_driver(tmp_path, oracle_only=False)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "RELAY DROPIN OK" in r.stdout


def _time_lines(out):
    import json
    rows = [json.loads(x) for x in out.splitlines() if x.startswith("{")]
    for r in rows:
        assert r["us_per_seq"]["chain"] > 0 and r["us_per_seq"]["relay_gf"] > 0, r
    return rows


def test_relay_driver_time_mode_over_oracle_methods(tmp_path):
    """relay_dropin_test.cpp --time P (the per-call cost of the relay class: slot shifts and GF calls
    per seq at the relay and the destination) runs over the oracle-method class on the CPU."""
    import subprocess
    exe = _build_relay_driver(tmp_path, oracle_only=True)
    r = subprocess.run([exe, "--time", "300"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert [(x["class"], x["type"]) for x in _time_lines(r.stdout)] == [("oracle", 2), ("oracle", 3)]


@pytest.mark.gpu
def test_gpu_relay_dropin_per_call_cost(tmp_path):
    """The per-call cost of siphon::Decoder_Symbol_Wise (every GF call a device round trip) beside
    the oracle-method class, per seq of a (10,3) relay chain; the lines are printed for the record
    (profiles/r05/relay/r05_per_call_relay.txt)."""
    import subprocess
    exe = _build_relay_driver(tmp_path, oracle_only=False)
    r = subprocess.run([exe, "--time", "3000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    rows = _time_lines(r.stdout)
    assert [(x["class"], x["type"]) for x in rows] == [("dropin", 2), ("dropin", 3), ("oracle", 2), ("oracle", 3)]
    print(r.stdout)


def _vr_relay_schedule(tmp_path, P):
    """Switch points and codes of config 4's schedule on bin/erasure.bin (the plan's encoder
    instances: each starts at its first seq), hop-1 erasures from bin/erasure.bin and hop-2 ones
    from bin/erasure2.bin, written for tests/cpp/relay_dropin_test.cpp --schedule."""
    import numpy as np
    from fec_erasure_code_unit_test_relay_amd.vr import VrPlan
    v = VrPlan(load_pattern("bin_erasure"), P)
    sched = []
    for T, B, N, first, _sw, _end in v.encoders.tolist():
        if first >= P:
            break
        assert B == N  # adaptive tuples are (T, N, N): the relay's source code
        if not sched or first >= sched[-1][0] + 11:  # T_TOT + 1 packets of double coding
            sched.append((first, T, N))
    f = tmp_path / "sched.txt"
    f.write_text(f"{P}\n" + "".join(f"{s} {T} {N}\n" for s, T, N in sched))
    e1, e2 = tmp_path / "e1.bin", tmp_path / "e2.bin"
    np.ascontiguousarray(load_pattern("bin_erasure")[:P], dtype=np.uint8).tofile(e1)
    np.ascontiguousarray(load_pattern("bin_erasure2")[:P], dtype=np.uint8).tofile(e2)
    return [str(f), str(e1), str(e2)], len(sched)


def test_relay_driver_vr_schedule_over_oracle_methods(tmp_path):
    """The relay driver through config 4's code switches on bin/erasure.bin (a relay under
    variable rate: double coding at every switch, Variable_Rate_FEC_Decoder.cpp:1423-1600,
    :1772-1873) over the oracle's per-call methods: runs clean (the GPU test compares the drop-in
    class with it seq by seq)."""
    import subprocess
    exe = _build_relay_driver(tmp_path, oracle_only=True)
    files, nsw = _vr_relay_schedule(tmp_path, 4000)
    assert nsw > 10
    r = subprocess.run([exe, "--schedule"] + files, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "RELAY ORACLE DRIVER OK" in r.stdout


@pytest.mark.gpu
def test_gpu_relay_dropin_vr_schedule_equals_oracle_methods(tmp_path):
    """siphon::Decoder_Symbol_Wise (GF work on the GPU) through config 4's code switches on
    bin/erasure.bin, types 2 and 3: every relay frame, destination output and flag equal to the
    oracle-method class's, seq by seq (12 000 seqs, ~60 double-coding transitions)."""
    import subprocess
    exe = _build_relay_driver(tmp_path, oracle_only=False)
    files, nsw = _vr_relay_schedule(tmp_path, 12000)
    assert nsw > 40
    r = subprocess.run([exe, "--schedule"] + files, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "RELAY DROPIN OK" in r.stdout


def test_relay_c_abi_rejects_bad_arguments_before_device_work():
    """The drop-in relay's per-call methods (fec_sw_*, include/fec_amd.h) and fec_sdswdf_create
    check their arguments before any HIP call (so this runs on the CPU): FEC_ERR_ARG for a missing
    array, k2 != k (the reference always calls them with k2 = k, Variable_Rate_FEC_Decoder.cpp:998),
    n2 < k, the state-dependent pair's n2 > n or n past T_TOT + 1, k < 1, max_payload < 1."""
    import ctypes
    from fec_erasure_code_unit_test_relay_amd._lib import lib
    Lb = lib()
    i, vp = ctypes.c_int, ctypes.c_void_p
    Lb.fec_sw_state_encode.argtypes = [i] * 6 + [vp] * 5
    Lb.fec_sw_state_decode.argtypes = [i] * 3 + [vp] * 4
    Lb.fec_sw_encode_1.argtypes = [i] * 5 + [vp] * 5
    Lb.fec_sw_decode_1.argtypes = [i] * 3 + [vp] * 4
    Lb.fec_sdswdf_create.argtypes = [i] * 6 + [ctypes.POINTER(vp)]
    buf = np.zeros(64, dtype=np.uint64)
    p = buf.ctypes.data_as(vp)
    ERR = -1
    for args in [(300, 8, 11, 7, 11, 0), (300, 8, 11, 8, 12, 0), (300, 8, 12, 8, 12, 0), (300, 0, 11, 0, 11, 0),
                 (300, 1, 4, 1, 1, 0)]:
        assert Lb.fec_sw_state_encode(*args, p, p, p, p, p) == ERR, args  # n2 <= n <= T_TOT + 1
    for args in [(300, 8, 11, 7, 11), (300, 8, 11, 8, 7), (300, 0, 11, 0, 11), (0, 8, 11, 8, 11)]:
        assert Lb.fec_sw_encode_1(*args, p, p, p, p, p) == ERR, args  # n2 >= k2 = k
    assert Lb.fec_sw_state_encode(300, 8, 11, 8, 11, 0, None, p, p, p, p) == ERR
    assert Lb.fec_sw_encode_1(300, 8, 11, 8, 11, p, None, p, p, p) == ERR
    assert Lb.fec_sw_state_decode(300, 8, 12, p, p, p, p) == ERR
    assert Lb.fec_sw_state_decode(300, 8, 11, p, None, p, p) == ERR
    assert Lb.fec_sw_decode_1(300, 0, 11, p, p, p, p) == ERR
    assert Lb.fec_sw_decode_1(0, 8, 11, p, p, p, p) == ERR
    h = vp()
    assert Lb.fec_sdswdf_create(300, 10, 3, 10, 4, 0, ctypes.byref(h)) == ERR  # k2 != k
    assert Lb.fec_sdswdf_create(300, 9, 3, 10, 4, 0, ctypes.byref(h)) == ERR   # T2 > T1
    assert Lb.fec_sdswdf_create(300, 3, 3, 0, 0, 0, ctypes.byref(h)) == ERR    # n2 = 1
    Lb.fec_swdf_create.argtypes = [i] * 5 + [ctypes.POINTER(vp)]
    assert Lb.fec_swdf_create(300, 3, 3, 0, 0, ctypes.byref(h)) == ERR         # n2 = 1


def _relay_vr_golden():
    import json
    import os
    from conftest import ROOT
    with open(os.path.join(ROOT, "tests", "golden", "relay_vr_360k.json")) as f:
        return json.load(f)


def test_relay_vr_golden_prefix_from_driver(tmp_path):
    """tests/golden/relay_vr_360k.json (made by tests/golden/make_relay_vr_golden.py from the
    reference-structured driver over the oracle's methods, all 360 000 seqs): the same driver on
    the first 3 000 seqs of its schedule reproduces its first 30 block digests (the chain is
    causal: a shorter run is a prefix)."""
    import subprocess
    import numpy as np
    g = _relay_vr_golden()
    exe = _build_relay_driver(tmp_path, oracle_only=True)
    P = 3000
    sched = [s for s in g["schedule"] if s[0] < P]
    f = tmp_path / "sched.txt"
    f.write_text(f"{P}\n" + "".join(f"{s} {T} {N}\n" for s, T, N in sched))
    e1, e2, dig = tmp_path / "e1.bin", tmp_path / "e2.bin", tmp_path / "dig.txt"
    np.ascontiguousarray(load_pattern("bin_erasure")[:P], dtype=np.uint8).tofile(e1)
    np.ascontiguousarray(load_pattern("bin_erasure2")[:P], dtype=np.uint8).tofile(e2)
    r = subprocess.run([exe, "--schedule", str(f), str(e1), str(e2), "--digest", str(dig)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = dig.read_text().split("\n")
    for t in ("2", "3"):
        i = next(j for j, ln in enumerate(lines) if ln.startswith(f"type {t} "))
        blocks = [ln.strip() for ln in lines[i + 1:i + 1 + P // 100]]
        assert blocks == g[f"type{t}"]["blocks"][:P // 100], t


def test_relay_vr_create_rejects_bad_schedules():
    """fec_relay_vr_create checks its schedule before any device work: relay type 2 or 3, the
    first switch at seq 0, switches at least T_TOT + 1 apart (one double-coding transition at a
    time, Variable_Rate_FEC_Encoder.cpp:74-235), 1 <= T <= T_TOT, 0 <= N <= T, seqs inside [0, P)."""
    import ctypes
    import numpy as np
    from fec_erasure_code_unit_test_relay_amd._lib import lib
    L = lib()
    h = ctypes.c_void_p()
    for typ, sched, P in [(1, [(0, 10, 3)], 100), (2, [(1, 10, 3)], 100), (3, [(0, 10, 3), (10, 10, 5)], 100),
                          (2, [(0, 11, 3)], 100), (2, [(0, 10, 11)], 100), (2, [(0, 0, 0)], 100),
                          (3, [(0, 10, 3), (100, 10, 5)], 100), (2, [(0, 10, 3)], 0)]:
        a = np.ascontiguousarray(np.asarray(sched, dtype=np.int32))
        st = L.fec_relay_vr_create(typ, 300, a.ctypes.data_as(ctypes.c_void_p), a.shape[0], P, ctypes.byref(h))
        assert st == -1, (typ, sched, P)


@pytest.mark.gpu
@pytest.mark.parametrize("relay_type", [2, 3])
def test_gpu_relay_vr_full_schedule_equals_driver(relay_type):
    """The batched relay chain under variable rate (fec_relay_vr: every code instance of config 4's
    schedule on bin/erasure.bin, hop 2 on bin/erasure2.bin, one fixed-rate batch per code with
    the instances end to end) equals, seq by seq, the reference-structured driver over the oracle's
    Decoder_Symbol_Wise methods for all 360 000 seqs: every frame (double-coding layout), every
    destination output and loss flag, by the golden file's per-100-seq CRC-32 digests.  The golden
    file (tests/golden/relay_vr_360k.json, make_relay_vr_golden.py) comes from this repo's oracle
    driver, not from reference output (the reference ships none): parity unpinned.  The frame
    layout through a switch is hand-traced in test_session.py::test_hop1_burst_then_adaptation."""
    import torch
    from fec_erasure_code_unit_test_relay_amd import fill_payload
    from fec_erasure_code_unit_test_relay_amd.relay import AdaptiveRelay, relay_digest
    torch.cuda.set_device(0)
    g = _relay_vr_golden()
    P = g["P"]
    r = AdaptiveRelay(relay_type, 300, g["schedule"], P)
    payload = fill_payload(0, P, 300, 0x5EED)
    frames, flen, out, flags = r.run(payload, load_pattern("bin_erasure"), load_pattern("bin_erasure2"))
    torch.cuda.synchronize()
    want = g[f"type{relay_type}"]
    assert int((flags == 0).sum()) == want["unflagged"]
    got = [f"{c:08x}" for c in relay_digest(frames, flen, out, flags)]
    bad = [i for i, (a, b) in enumerate(zip(got, want["blocks"])) if a != b]
    assert len(got) == len(want["blocks"]) and not bad, f"first differing block {bad[:5]} of {len(got)}"
