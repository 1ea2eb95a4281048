"""oracle -- TEST INFRASTRUCTURE ONLY (the checker, never the product).

ctypes loader for the plain-C restatement in ``oracle/fec_oracle.c`` of the reference's GF(2^8)
streaming-erasure hot path (domanovi/FEC_Erasure_Code_Unit_Test_Relay: src/basicOperations.cpp,
src/codingOperations.cpp, src/Encoder*.cpp, src/Decoder*.cpp, src/FEC_Encoder.cpp,
src/FEC_Decoder.cpp).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module.  The reference itself is unbuildable here (it needs
Intel ISA-L, which is absent); the restatement is pinned by the reference's published fixed-rate
loss counts (tests/golden/published_fixed_logs.json).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    """Compile the restatement with gcc (oracle/Makefile) and return the .so path."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        src = os.path.join(_HERE, "fec_oracle.c")
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        ip = ctypes.POINTER(ctypes.c_int)
        L.or_gf_mul.restype = ctypes.c_uint8
        L.or_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.or_gf_inv.restype = ctypes.c_uint8
        L.or_gf_inv.argtypes = [ctypes.c_uint8]
        L.or_gen_G.argtypes = [u8p] + [ctypes.c_int] * 5
        L.or_rref_matrix.argtypes = [u8p, u8p, u8p, ctypes.c_int, ctypes.c_int]
        L.or_decode_block.argtypes = [u8p, u8p, u8p, u8p] + [ctypes.c_int] * 4
        L.or_encode_block.argtypes = [u8p, u8p, u8p] + [ctypes.c_int] * 3
        L.or_geometry.argtypes = [ctypes.c_int] * 4 + [ip] * 4
        L.or_encoder_new.restype = ctypes.c_void_p
        L.or_encoder_new.argtypes = [ctypes.c_int] * 4
        L.or_encoder_free.argtypes = [ctypes.c_void_p]
        L.or_encoder_transmit.restype = ctypes.c_int
        L.or_encoder_transmit.argtypes = [ctypes.c_void_p, u8p, ctypes.c_int, ctypes.c_int, u8p]
        L.or_decoder_new.restype = ctypes.c_void_p
        L.or_decoder_new.argtypes = [ctypes.c_int] * 5
        L.or_decoder_free.argtypes = [ctypes.c_void_p]
        L.or_decoder_receive.restype = ctypes.c_int
        L.or_decoder_receive.argtypes = [ctypes.c_void_p, u8p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, u8p]
        L.or_fill_payload.argtypes = [u8p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                      ctypes.c_uint64]
        L.or_run_stream.restype = ctypes.c_int64
        L.or_run_stream.argtypes = [ctypes.c_int] * 4 + [ctypes.c_int64, u8p, ctypes.c_int64,
                                    ctypes.c_uint64, ctypes.c_int, ip, u8p, u8p, ip]
        L.or_encode_stream.restype = ctypes.c_int64
        L.or_encode_stream.argtypes = [ctypes.c_int] * 4 + [ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_uint64, u8p, ip]
        L.or_swdf_run.restype = ctypes.c_int
        L.or_swdf_run.argtypes = [ctypes.c_int] * 5 + [ctypes.c_int64, u8p, u8p, ctypes.c_uint64,
                                                        u8p, u8p, u8p, u8p]
        L.or_sdswdf_run.restype = ctypes.c_int
        L.or_sdswdf_run.argtypes = [ctypes.c_int] * 5 + [ctypes.c_int64, u8p, u8p, ctypes.c_uint64,
                                                          ctypes.c_int, u8p, u8p, u8p]
        L.or_sdswdf_set_garbage.argtypes = [ctypes.c_int]
        L.or_vr_run.restype = ctypes.c_int64
        i64p = ctypes.POINTER(ctypes.c_int64)
        L.or_vr_run.argtypes = [ctypes.c_int] * 5 + [u8p, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64, ip,
                                                      u8p, u8p, ctypes.c_int64, i64p, ctypes.c_int64,
                                                      i64p, ctypes.POINTER(ctypes.c_double)]
        L.or_relay_session_run.restype = ctypes.c_int
        L.or_relay_session_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, u8p, ctypes.c_int64, u8p,
                                           ctypes.c_int64, ctypes.c_uint64, ctypes.POINTER(SessionOut)]
        _lib = L
    return _lib


SESSION_DW = 320      # OR_SESSION_DW
SESSION_BLOCK = 100   # OR_SESSION_BLOCK


class SessionOut(ctypes.Structure):
    """or_session_out (oracle/fec_oracle.h)."""
    _fields_ = [("Q", ctypes.c_int64)] + [(f, ctypes.c_void_p) for f in (
        "hop1_len", "hop1_hdr", "relay_len", "relay_hdr", "dest_proc", "dest_flag", "dest_lost", "dest_out",
        "crc", "crc2", "hop1_pkts", "relay_pkts")] + [
        ("hop1_stride", ctypes.c_int64), ("relay_stride", ctypes.c_int64)] + [(f, ctypes.c_int64) for f in (
            "lost", "src_switches", "relay_switches", "dest_switches", "relay_flags", "dest_flags",
            "status_seq")] + [(f, ctypes.c_float) for f in ("rate1", "rate2", "min_rate")] + [
        (f, ctypes.c_int64) for f in ("rate1_n", "rate2_n", "min_rate_n")]


def _u8(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _i32(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def geometry(max_payload: int, T: int, B: int, N: int):
    """(k, n, S, CW) exactly as Encoder.cpp:31-39 derives them."""
    v = [ctypes.c_int() for _ in range(4)]
    lib().or_geometry(max_payload, T, B, N, *[ctypes.byref(x) for x in v])
    return tuple(x.value for x in v)


def gf_mul(a: int, b: int) -> int:
    return int(lib().or_gf_mul(a, b))


def gf_inv(a: int) -> int:
    return int(lib().or_gf_inv(a))


def gen_G(T: int, B: int, N: int) -> np.ndarray:
    """k x n generator matrix (gen_G_cauchy, codingOperations.cpp:48-95)."""
    k, n = T - N + 1, T - N + 1 + B
    G = np.zeros(k * n, dtype=np.uint8)
    lib().or_gen_G(_u8(G), T, B, N, k, n)
    return G.reshape(k, n)


def rref(mat: np.ndarray):
    """gf256_rref_matrix (basicOperations.cpp:43-122) -> (out, action)."""
    m, n = mat.shape
    inp = np.ascontiguousarray(mat, dtype=np.uint8)
    out = np.zeros_like(inp)
    act = np.zeros((n, n), dtype=np.uint8)
    lib().or_rref_matrix(_u8(inp), _u8(out), _u8(act), m, n)
    return out, act


def encode_block(data: np.ndarray, G: np.ndarray, cw: np.ndarray, t: int) -> np.ndarray:
    """encodeBlock (codingOperations.cpp:131-147) on one block; cw is updated in place."""
    k, n = G.shape
    d = np.ascontiguousarray(data, dtype=np.uint8)
    g = np.ascontiguousarray(G, dtype=np.uint8)
    lib().or_encode_block(_u8(d), _u8(g), _u8(cw), k, n, t)
    return cw


def decode_block(cw: np.ndarray, G: np.ndarray, erasure: np.ndarray, T: int, t: int):
    """decodeBlock (codingOperations.cpp:149-232) in the relay's in-place form
    decodeBlock(cw, G, cw, erasure, k, n, T, t); returns (cw, erasure) updated."""
    k, n = G.shape
    c = np.array(cw, dtype=np.uint8)
    e = np.array(erasure, dtype=np.uint8)
    g = np.ascontiguousarray(G, dtype=np.uint8)
    lib().or_decode_block(_u8(c), _u8(g), _u8(c), _u8(e), k, n, T, t)
    return c, e


def fill_payload(t0: int, count: int, L: int, seed: int) -> np.ndarray:
    """Synthetic payloads: byte b of packet t = splitmix64(seed ^ (t*L + b)) & 0xff."""
    buf = np.zeros(count * L, dtype=np.uint8)
    lib().or_fill_payload(_u8(buf), t0, count, L, seed)
    return buf.reshape(count, L)


class Encoder:
    """FEC_Encoder (src/FEC_Encoder.cpp:22-68) as restated by the oracle."""

    def __init__(self, max_payload: int, T: int, B: int, N: int):
        self.L = max_payload
        self.k, self.n, self.S, self.CW = geometry(max_payload, T, B, N)
        self._h = lib().or_encoder_new(max_payload, T, B, N)
        if not self._h:
            raise ValueError("unsupported (T,B,N)")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_encoder_free(self._h)
            self._h = None

    def onTransmit(self, data: np.ndarray, payload: int, seq: int):
        """Returns (untrimmed CW-byte codeword, trimmed wire size)."""
        d = np.ascontiguousarray(data, dtype=np.uint8)
        cw = np.zeros(self.CW, dtype=np.uint8)
        size = lib().or_encoder_transmit(self._h, _u8(d), payload, seq, _u8(cw))
        return cw, size


class Decoder:
    """FEC_Decoder (src/FEC_Decoder.cpp:26-72) as restated by the oracle."""

    def __init__(self, max_payload: int, T: int, B: int, N: int, loss_only: bool = False):
        self.L = max_payload
        self.k, self.n, self.S, self.CW = geometry(max_payload, T, B, N)
        self._h = lib().or_decoder_new(max_payload, T, B, N, int(loss_only))
        if not self._h:
            raise ValueError("unsupported (T,B,N)")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_decoder_free(self._h)
            self._h = None

    def onReceive(self, codeword, size: int, seq: int, erasure: bool):
        """Returns (max_payload bytes of packet seq-T zero-filled past the payload, payload length)."""
        out = np.zeros(self.L, dtype=np.uint8)
        if erasure or codeword is None:
            p = lib().or_decoder_receive(self._h, None, 0, seq, 1, _u8(out))
        else:
            c = np.ascontiguousarray(codeword, dtype=np.uint8)
            p = lib().or_decoder_receive(self._h, _u8(c), size, seq, 0, _u8(out))
        return out, p


def run_stream(max_payload: int, T: int, B: int, N: int, P: int, pattern: np.ndarray,
               seed: int = 0x5EED, loss_only: bool = False, want_data: bool = False,
               want_codewords: bool = False):
    """Feed seq 0..P+T-1 through FEC_Encoder -> erasure channel -> FEC_Decoder.

    Returns dict(lost, out_len[P], out_data[P,L]?, cw[P+T,CW]?, cw_len[P+T]?).
    """
    k, n, S, CW = geometry(max_payload, T, B, N)
    pat = np.ascontiguousarray(pattern, dtype=np.uint8)
    out_len = np.zeros(P, dtype=np.int32)
    out_data = np.zeros((P, max_payload), dtype=np.uint8) if want_data else None
    cw = np.zeros((P + T, CW), dtype=np.uint8) if want_codewords else None
    cw_len = np.zeros(P + T, dtype=np.int32) if want_codewords else None
    lost = lib().or_run_stream(max_payload, T, B, N, P, _u8(pat), pat.size, seed, int(loss_only),
                               _i32(out_len), _u8(out_data) if want_data else None,
                               _u8(cw) if want_codewords else None,
                               _i32(cw_len) if want_codewords else None)
    if lost < 0:
        raise ValueError("unsupported (T,B,N)")
    return dict(lost=int(lost), out_len=out_len, out_data=out_data, cw=cw, cw_len=cw_len)


def encode_stream(max_payload: int, T: int, B: int, N: int, seq0: int, P: int, seed: int = 0x5EED,
                  want_codewords: bool = True):
    k, n, S, CW = geometry(max_payload, T, B, N)
    cw = np.zeros((P, CW), dtype=np.uint8) if want_codewords else None
    cw_len = np.zeros(P, dtype=np.int32) if want_codewords else None
    total = lib().or_encode_stream(max_payload, T, B, N, seq0, P, seed,
                                   _u8(cw) if want_codewords else None,
                                   _i32(cw_len) if want_codewords else None)
    return dict(total=int(total), cw=cw, cw_len=cw_len)


def swdf_run(max_payload: int, T1: int, N1: int, T2: int, N2: int, P: int, e1: np.ndarray,
             e2: np.ndarray, seed: int = 0x5EED):
    """The local simulation's SWDF chain (source FEC_Encoder -> hop 1 -> relay
    Decoder_Symbol_Wise::symbol_wise_encode_1 -> hop 2 -> destination symbol_wise_decode_1 +
    extract_data, one relay frame per seq): returns dict(frames [P, 2+(S+1)*n2], relay_flag [P],
    dest_out [P, S*k] (data_with_header), dest_flag [P], delay = n1+n2-k-1)."""
    k, n1, n2 = T1 - N1 + 1, T1 + 1, T2 + 1
    S = -(-(max_payload + 2) // k)
    F = 2 + (S + 1) * n2
    a = np.ascontiguousarray(e1[:P], dtype=np.uint8)
    b = np.ascontiguousarray(e2[:P], dtype=np.uint8)
    assert a.size == P and b.size == P
    frames = np.zeros((P, F), dtype=np.uint8)
    rf = np.zeros(P, dtype=np.uint8)
    out = np.zeros((P, S * k), dtype=np.uint8)
    df = np.zeros(P, dtype=np.uint8)
    st = lib().or_swdf_run(max_payload, T1, N1, T2, N2, P, _u8(a), _u8(b), seed, _u8(frames), _u8(rf),
                           _u8(out), _u8(df))
    if st != 0:
        raise ValueError("unsupported SWDF configuration")
    return dict(frames=frames, relay_flag=rf, dest_out=out, dest_flag=df, delay=n1 + n2 - k - 1, S=S, k=k)


def sdswdf_run(max_payload: int, T1: int, N1: int, T2: int, N2: int, P: int, e1: np.ndarray,
               e2: np.ndarray, seed: int = 0x5EED, sdbo: int = 0, garbage: int = 0):
    """The local simulation's state-dependent SWDF chain (RELAYING_TYPE 3, one relay frame per seq):
    source FEC_Encoder -> hop 1 -> relay symbol_wise_encode_state_dependent -> hop 2 -> destination
    symbol_wise_decode_state_dependent + extract_data.  Returns dict(frames [P, 2+11+(S+1)*n2],
    dest_out [P, S*k] (data_with_header), dest_flag [P], delay = n1+n2-k-1).  `garbage` is the
    relay's temp_codeword content at the start of each call (outputs must not depend on it)."""
    k, n1, n2 = T1 - N1 + 1, T1 + 1, T2 + 1
    S = -(-(max_payload + 2) // k)
    F = 2 + 11 + (S + 1) * n2
    a = np.ascontiguousarray(e1[:P], dtype=np.uint8)
    b = np.ascontiguousarray(e2[:P], dtype=np.uint8)
    assert a.size == P and b.size == P
    frames = np.zeros((P, F), dtype=np.uint8)
    out = np.zeros((P, S * k), dtype=np.uint8)
    df = np.zeros(P, dtype=np.uint8)
    lib().or_sdswdf_set_garbage(garbage)
    st = lib().or_sdswdf_run(max_payload, T1, N1, T2, N2, P, _u8(a), _u8(b), seed, sdbo, _u8(frames),
                             _u8(out), _u8(df))
    lib().or_sdswdf_set_garbage(0)
    if st != 0:
        raise ValueError("unsupported SD-SWDF configuration")
    return dict(frames=frames, dest_out=out, dest_flag=df, delay=n1 + n2 - k - 1, S=S, k=k)


def vr_run(pattern: np.ndarray, P: int, max_payload: int = 300, T: int = 10, B: int = -1, N: int = -1,
           mds: bool = False, seed: int = 0x5EED, want_data: bool = False, max_sent: int = 0,
           packets_cap: int = 0):
    """The adaptive P2P loop (sender -> Variable_Rate_FEC_Encoder -> erasure -> receiver with its
    Parameter_Estimator pair -> Variable_Rate_FEC_Decoder), reference-structured on real bytes.
    Returns dict(lost, switches, sent, coding_rate, out_len [P], out_data?, packets?, packet_off?):
    packets = the first max_sent P2P wire packets back to back, packet_off their offsets."""
    pat = np.ascontiguousarray(pattern, dtype=np.uint8)
    out_len = np.zeros(P, dtype=np.int32)
    out_data = np.zeros((P, max_payload), dtype=np.uint8) if want_data else None
    packets = np.zeros(packets_cap, dtype=np.uint8) if packets_cap else None
    packet_off = np.zeros(max_sent + 1, dtype=np.int64) if max_sent else None
    stats = (ctypes.c_int64 * 3)()
    rate = ctypes.c_double()
    lib().or_vr_run(max_payload, T, B, N, int(mds), _u8(pat), pat.size, P, seed, _i32(out_len),
                    _u8(out_data) if want_data else None, _u8(packets) if packets_cap else None, packets_cap,
                    packet_off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)) if max_sent else None, max_sent,
                    stats, ctypes.byref(rate))
    res = dict(lost=int(stats[0]), switches=int(stats[1]), sent=int(stats[2]), coding_rate=rate.value,
               out_len=out_len, out_data=out_data, packets=None, packet_off=packet_off)
    if packets_cap:
        assert packet_off[-1] <= packets_cap, "packets_cap too small"
        res["packets"] = packets[: packet_off[-1]]
    return res


def relay_session_run(relay_type: int, Q: int, e1: np.ndarray, e2: np.ndarray, max_payload: int = 300,
                      seed: int = 0x5EED, want_out: bool = False, hop1_stride: int = 0, relay_stride: int = 0):
    """The two-hop adaptive relay session (RELAYING_TYPE 2 / 3, application_local_simulation.cpp:71-593
    with constant transmission) for Q seqs over hop patterns e1 / e2: the reference-structured
    oracle loop (or_relay_session_run).  Returns dict(lost, switches (source, relay, destination),
    rates, hop1_len / relay_len [Q], hop1_hdr [Q,16], relay_hdr [Q,8], crc / crc2 per block of
    SESSION_BLOCK seqs, and with want_out dest_proc / dest_flag / dest_lost [Q], dest_out [Q,
    SESSION_DW]; hop1_pkts / relay_pkts [Q, stride] when a stride is given)."""
    a = np.ascontiguousarray(e1, dtype=np.uint8)
    b = np.ascontiguousarray(e2, dtype=np.uint8)
    nb = (Q + SESSION_BLOCK - 1) // SESSION_BLOCK
    r = dict(hop1_len=np.zeros(Q, np.int32), hop1_hdr=np.zeros((Q, 16), np.uint8), relay_len=np.zeros(Q, np.int32),
             relay_hdr=np.zeros((Q, 8), np.uint8), crc=np.zeros(nb, np.uint32))
    if want_out:
        r.update(dest_proc=np.zeros(Q, np.uint8), dest_flag=np.zeros(Q, np.uint8), dest_lost=np.zeros(Q, np.uint8),
                 dest_out=np.zeros((Q, SESSION_DW), np.uint8), crc2=np.zeros(nb, np.uint32))
    if hop1_stride:
        r["hop1_pkts"] = np.zeros((Q, hop1_stride), np.uint8)
    if relay_stride:
        r["relay_pkts"] = np.zeros((Q, relay_stride), np.uint8)
    o = SessionOut()
    o.hop1_stride, o.relay_stride = hop1_stride, relay_stride
    for f, v in r.items():
        setattr(o, f, v.ctypes.data)
    rc = lib().or_relay_session_run(relay_type, max_payload, Q, _u8(a), a.size, _u8(b), b.size, seed, ctypes.byref(o))
    if rc != 0:
        raise ValueError(f"or_relay_session_run: {rc} at seq {o.status_seq}")
    r.update(lost=o.lost, src_switches=o.src_switches, relay_switches=o.relay_switches,
             dest_switches=o.dest_switches, relay_flags=o.relay_flags, dest_flags=o.dest_flags,
             rate1=o.rate1, rate1_n=o.rate1_n, rate2=o.rate2, rate2_n=o.rate2_n, min_rate=o.min_rate,
             min_rate_n=o.min_rate_n)
    return r
