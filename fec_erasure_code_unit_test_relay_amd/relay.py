"""Relay symbol-wise decode-and-forward (SWDF) over the MI355X C ABI (include/fec_amd.h,
fec_swdf_*).

Mirrors what Decoder_Symbol_Wise (src/Decoder_Symbol_Wise.cpp) does at the relay
(``symbol_wise_encode_1`` after ``push_current_codeword`` / ``rotate_pointers_and_insert_zero_word``,
driven by Variable_Rate_FEC_Decoder::receive_message_and_symbol_wise_encode, :950-1601) and at the
destination (``symbol_wise_decode_1`` + ``extract_data``, :1603-1879), batched over many packets
of one relay stream held in HBM.
"""
from __future__ import annotations

import ctypes

from ._lib import check, lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class SymbolWiseRelay:
    """Fixed-rate SWDF chain: source (T1, N1, N1) -> relay -> destination with (T2, N2), where
    k = T1-N1+1 = T2-N2+1 (the relay keeps the data symbols and changes the code length)."""

    def __init__(self, max_payload: int, T1: int, N1: int, T2: int, N2: int):
        h = ctypes.c_void_p()
        check(lib().fec_swdf_create(max_payload, T1, N1, T2, N2, ctypes.byref(h)), "fec_swdf_create")
        self._h = h
        v = [ctypes.c_int() for _ in range(6)]
        check(lib().fec_swdf_geometry(h, *[ctypes.byref(x) for x in v]), "fec_swdf_geometry")
        self.k, self.n1, self.n2, self.S, self.frame_bytes, self.delay = (x.value for x in v)
        self.L = max_payload
        self._work = None

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                lib().fec_swdf_destroy(self._h)
            except Exception:
                pass
            self._h = None

    def relay(self, codewords, erasure, frames=None, flag=None):
        """symbol_wise_encode_1 for seqs 0..P-1: source codewords [P, >= S*n1] uint8 (zero-padded
        rows) and hop-1 erasure flags [P] -> (frames [P, frame_bytes], flags [P] uint8)."""
        import torch
        assert codewords.dtype == torch.uint8 and codewords.is_cuda and codewords.is_contiguous()
        assert codewords.dim() == 2 and codewords.shape[1] >= self.S * self.n1
        P = codewords.shape[0]
        assert erasure.dtype == torch.uint8 and erasure.is_cuda and erasure.is_contiguous() and erasure.numel() >= P
        if frames is None:
            frames = torch.empty((P, self.frame_bytes), dtype=torch.uint8, device=codewords.device)
        assert frames.shape == (P, self.frame_bytes) and frames.is_contiguous() and frames.dtype == torch.uint8
        if flag is None:
            flag = torch.empty(P, dtype=torch.uint8, device=codewords.device)
        assert flag.numel() >= P and flag.dtype == torch.uint8 and flag.is_contiguous()
        nbytes = int(lib().fec_swdf_workspace_bytes(self._h, P))
        if self._work is None or self._work.numel() < nbytes:
            self._work = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=codewords.device)
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        check(lib().fec_swdf_relay_batch(self._h, _ptr(codewords), codewords.shape[1], _ptr(erasure), P,
                                         _ptr(frames), _ptr(flag), _ptr(self._work), self._work.numel(),
                                         stream), "fec_swdf_relay_batch")
        return frames, flag

    def destination(self, frames, erasure, out=None, flag=None):
        """symbol_wise_decode_1 + extract_data for seqs 0..P-1: relay frames [P, frame_bytes] and
        hop-2 erasure flags [P] -> (data_with_header rows [P, S*k] (row t = source packet
        t - delay), flags [P] uint8)."""
        import torch
        assert frames.dtype == torch.uint8 and frames.is_cuda and frames.is_contiguous()
        assert frames.dim() == 2 and frames.shape[1] == self.frame_bytes
        P = frames.shape[0]
        assert erasure.dtype == torch.uint8 and erasure.is_cuda and erasure.is_contiguous() and erasure.numel() >= P
        if out is None:
            out = torch.empty((P, self.S * self.k), dtype=torch.uint8, device=frames.device)
        assert out.shape == (P, self.S * self.k) and out.is_contiguous() and out.dtype == torch.uint8
        if flag is None:
            flag = torch.empty(P, dtype=torch.uint8, device=frames.device)
        assert flag.numel() >= P and flag.dtype == torch.uint8 and flag.is_contiguous()
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        check(lib().fec_swdf_destination_batch(self._h, _ptr(frames), _ptr(erasure), P, _ptr(out), _ptr(flag),
                                               stream), "fec_swdf_destination_batch")
        return out, flag


class StateDependentRelay:
    """Fixed-rate SD-SWDF chain (RELAYING_TYPE 3): source (T1, N1, N1) -> relay
    (symbol_wise_encode_state_dependent, Decoder_Symbol_Wise.cpp:178-432) -> destination
    (symbol_wise_decode_state_dependent + extract_data, :487-546, :653-661), with
    k = T1-N1+1 = T2-N2+1 and T2 <= T1 <= T_TOT = 10.  The erasure flags of both hops are host
    arrays: they drive the host planner (the reference's per-packet control flow); the bytes stay
    on the GPU."""

    RECORD_HDR = 11

    def __init__(self, max_payload: int, T1: int, N1: int, T2: int, N2: int, sdbo: int = 0):
        h = ctypes.c_void_p()
        check(lib().fec_sdswdf_create(max_payload, T1, N1, T2, N2, sdbo, ctypes.byref(h)), "fec_sdswdf_create")
        self._h = h
        v = [ctypes.c_int() for _ in range(7)]
        check(lib().fec_sdswdf_geometry(h, *[ctypes.byref(x) for x in v]), "fec_sdswdf_geometry")
        self.k, self.n1, self.n2, self.S, self.blocks, self.frame_bytes, self.delay = (x.value for x in v)
        self.L = max_payload

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                lib().fec_sdswdf_destroy(self._h)
            except Exception:
                pass
            self._h = None

    @staticmethod
    def _host_flags(erasure, P):
        import numpy as np
        e = np.ascontiguousarray(np.asarray(erasure)[:P], dtype=np.uint8)
        assert e.size == P
        return e

    def relay(self, codewords, erasure, frames=None):
        """seqs 0..P-1: source codewords [P, >= S*n1] uint8 on the GPU (zero-padded rows; erased
        rows are never read), hop-1 flags [P] (host array) -> frames [P, frame_bytes]."""
        import torch
        assert codewords.dtype == torch.uint8 and codewords.is_cuda and codewords.is_contiguous()
        assert codewords.dim() == 2 and codewords.shape[1] >= self.S * self.n1
        P = codewords.shape[0]
        e = self._host_flags(erasure, P)
        if frames is None:
            frames = torch.empty((P, self.frame_bytes), dtype=torch.uint8, device=codewords.device)
        assert frames.shape == (P, self.frame_bytes) and frames.is_contiguous() and frames.dtype == torch.uint8
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        check(lib().fec_sdswdf_relay_batch(self._h, _ptr(codewords), codewords.shape[1],
                                           e.ctypes.data_as(ctypes.c_void_p), P, _ptr(frames), stream),
              "fec_sdswdf_relay_batch")
        return frames

    def destination(self, frames, erasure, out=None):
        """seqs 0..P-1: relay frames [P, frame_bytes] on the GPU, hop-2 flags [P] (host array) ->
        (data_with_header rows [P, S*k] on the GPU (row t = source packet t - delay), flags [P]
        numpy uint8)."""
        import numpy as np
        import torch
        assert frames.dtype == torch.uint8 and frames.is_cuda and frames.is_contiguous()
        assert frames.dim() == 2 and frames.shape[1] == self.frame_bytes
        P = frames.shape[0]
        e = self._host_flags(erasure, P)
        if out is None:
            out = torch.empty((P, self.S * self.k), dtype=torch.uint8, device=frames.device)
        assert out.shape == (P, self.S * self.k) and out.is_contiguous() and out.dtype == torch.uint8
        flag = np.zeros(P, dtype=np.uint8)
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        check(lib().fec_sdswdf_destination_batch(self._h, _ptr(frames), e.ctypes.data_as(ctypes.c_void_p), P,
                                                 _ptr(out), flag.ctypes.data_as(ctypes.c_void_p), stream),
              "fec_sdswdf_destination_batch")
        return out, flag

    def relay_plan(self, erasure):
        """The relay's host plan alone (no GPU): (record id per seq [P] int32, records [R, 11 +
        n2*n1] uint8: header bytes, then n2 rows of n1 coefficients)."""
        import numpy as np
        e = self._host_flags(erasure, len(erasure))
        P = e.size
        ids = np.zeros(P, dtype=np.int32)
        n = ctypes.c_int64()
        rb = ctypes.c_int()
        check(lib().fec_sdswdf_relay_plan(self._h, e.ctypes.data_as(ctypes.c_void_p), P,
                                          ids.ctypes.data_as(ctypes.c_void_p), None, 0, ctypes.byref(n),
                                          ctypes.byref(rb)), "fec_sdswdf_relay_plan")
        rec = np.zeros((n.value, rb.value), dtype=np.uint8)
        check(lib().fec_sdswdf_relay_plan(self._h, e.ctypes.data_as(ctypes.c_void_p), P,
                                          ids.ctypes.data_as(ctypes.c_void_p), rec.ctypes.data_as(ctypes.c_void_p),
                                          rec.size, ctypes.byref(n), ctypes.byref(rb)), "fec_sdswdf_relay_plan")
        return ids, rec

    def dest_plan(self, erasure, headers):
        """The destination's host plan alone (no GPU): headers [P, 11] = bytes 2..12 of every
        frame -> (record id per seq, records [R, k*n2], flags [P])."""
        import numpy as np
        e = self._host_flags(erasure, len(erasure))
        P = e.size
        hd = np.ascontiguousarray(headers[:P], dtype=np.uint8)
        assert hd.shape == (P, 11)
        ids = np.zeros(P, dtype=np.int32)
        fl = np.zeros(P, dtype=np.uint8)
        n = ctypes.c_int64()
        rb = ctypes.c_int()
        args = [self._h, e.ctypes.data_as(ctypes.c_void_p), hd.ctypes.data_as(ctypes.c_void_p), P,
                ids.ctypes.data_as(ctypes.c_void_p), fl.ctypes.data_as(ctypes.c_void_p)]
        check(lib().fec_sdswdf_dest_plan(*args, None, 0, ctypes.byref(n), ctypes.byref(rb)), "fec_sdswdf_dest_plan")
        rec = np.zeros((n.value, rb.value), dtype=np.uint8)
        check(lib().fec_sdswdf_dest_plan(*args, rec.ctypes.data_as(ctypes.c_void_p), rec.size, ctypes.byref(n),
                                         ctypes.byref(rb)), "fec_sdswdf_dest_plan")
        return ids, rec, fl


T_TOT = 10  # FEC_Macro.h


class AdaptiveRelay:
    """The relay chain under variable rate (RELAYING_TYPE 2 or 3 through code switches,
    Variable_Rate_FEC_Decoder.cpp:600-740 relay, :1423-1600 / :1772-1873 destination), batched:
    ``schedule`` = [(seq, T, N), ...] source codes (T, N, N), the first at seq 0, each at least
    T_TOT + 1 after the previous (the T_TOT + 1 double-coded seqs of a switch); hop 2 re-encodes
    with the same (T, N).  ``run`` returns what the relay sends per seq ([BE16 size][new part]
    [old part during double coding]) and what the reporting destination object outputs per seq
    (fec_relay_vr_* in include/fec_amd.h)."""

    def __init__(self, relay_type: int, max_payload: int, schedule, P: int):
        import numpy as np
        sched = np.ascontiguousarray(np.asarray(schedule, dtype=np.int32).reshape(-1, 3))
        h = ctypes.c_void_p()
        check(lib().fec_relay_vr_create(relay_type, max_payload, sched.ctypes.data_as(ctypes.c_void_p), sched.shape[0],
                                        P, ctypes.byref(h)), "fec_relay_vr_create")
        self._h = h
        v = [ctypes.c_int() for _ in range(3)]
        check(lib().fec_relay_vr_geometry(h, *[ctypes.byref(x) for x in v]), "fec_relay_vr_geometry")
        self.frame_stride, self.out_stride, self.codes = (x.value for x in v)
        self.type, self.L, self.P = relay_type, max_payload, P

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                lib().fec_relay_vr_destroy(self._h)
            except Exception:
                pass
            self._h = None

    @staticmethod
    def schedule_from_plan(plan, P: int):
        """Switch points of a variable-rate plan's encoder instances (fec_vr.VrPlan.encoders:
        (T, B, N, first, role switch, end), adaptive tuples B = N) that start at least T_TOT + 1
        seqs after the previous kept one, as the relay's code schedule."""
        sched = []
        for T, B, N, first, _sw, _end in plan.encoders.tolist():
            if first >= P:
                break
            if not sched or first >= sched[-1][0] + T_TOT + 1:
                sched.append((int(first), int(T), int(N)))
        return sched

    def run(self, payload, e1, e2):
        """payload [P, L] uint8 on the GPU (source packet t), hop erasure flags e1 / e2 (P host
        bytes, numpy) -> (frames [P, frame_stride], frame_len [P] int32, out [P, out_stride], flags
        [P] numpy uint8)."""
        import numpy as np
        import torch
        assert payload.dtype == torch.uint8 and payload.is_cuda and payload.is_contiguous()
        assert tuple(payload.shape) == (self.P, self.L)
        e1 = np.ascontiguousarray(np.asarray(e1, dtype=np.uint8)[:self.P])
        e2 = np.ascontiguousarray(np.asarray(e2, dtype=np.uint8)[:self.P])
        assert e1.size == self.P and e2.size == self.P
        dev = payload.device
        frames = torch.empty((self.P, self.frame_stride), dtype=torch.uint8, device=dev)
        flen = torch.empty(self.P, dtype=torch.int32, device=dev)
        out = torch.empty((self.P, self.out_stride), dtype=torch.uint8, device=dev)
        flags = np.zeros(self.P, dtype=np.uint8)
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        check(lib().fec_relay_vr_run(self._h, _ptr(payload), e1.ctypes.data_as(ctypes.c_void_p),
                                     e2.ctypes.data_as(ctypes.c_void_p), _ptr(frames), _ptr(flen), _ptr(out),
                                     flags.ctypes.data_as(ctypes.c_void_p), stream), "fec_relay_vr_run")
        return frames, flen, out, flags


class RelaySession:
    """The two-hop adaptive relay session (RELAYING_TYPE 2 / 3 with N_INITIAL = N_INITIAL_2 = -1,
    application_local_simulation.cpp:71-593): source (Application_Layer_Sender with the relay's
    12-byte feedback, the relay-mode Variable_Rate_FEC_Encoder) -> hop 1 -> relay
    (receive_message_and_symbol_wise_encode + send_sym_wise_message) -> hop 2 -> destination
    (receive_message_and_symbol_wise_decode), for Q seqs over the hop patterns e1 / e2
    (fec_relay_session_* in include/fec_amd.h).  The control plane runs at construction (host, on
    the patterns alone); run() does the session's byte work on the GPU."""

    DW = 320  # destination output row

    def __init__(self, relay_type: int, Q: int, e1, e2, max_payload: int = 300):
        import numpy as np
        a = np.ascontiguousarray(np.asarray(e1, dtype=np.uint8))
        b = np.ascontiguousarray(np.asarray(e2, dtype=np.uint8))
        h = ctypes.c_void_p()
        check(lib().fec_relay_session_create(relay_type, max_payload, Q, a.ctypes.data_as(ctypes.c_void_p), a.size,
                                             b.ctypes.data_as(ctypes.c_void_p), b.size, ctypes.byref(h)),
              "fec_relay_session_create")
        self._h = h
        self.type, self.Q, self.L = relay_type, Q, max_payload
        st = np.zeros(16, np.int64)
        rt = np.zeros(4, np.float64)
        check(lib().fec_relay_session_info(h, st.ctypes.data_as(ctypes.c_void_p), rt.ctypes.data_as(ctypes.c_void_p)),
              "fec_relay_session_info")
        keys = ("Q", "relay_bytes", "src_switches", "relay_switches", "dest_switches", "dest_flags", "relay_calls",
                "lineages", "dest_outputs", "processed", "symbol_bytes", "encoder_instances", "longest_lineage",
                "relay_flags", "rate1_n", "rate2_n")
        self.stats = {k: int(v) for k, v in zip(keys, st)}
        self.stats.update(rate1=float(rt[0]), rate2=float(rt[1]), min_rate=float(rt[2]), control_ms=float(rt[3]))
        self.relay_off = np.zeros(Q + 1, np.int64)
        check(lib().fec_relay_session_relay_offsets(h, self.relay_off.ctypes.data_as(ctypes.c_void_p)),
              "fec_relay_session_relay_offsets")
        self.hop1_hdr = np.zeros((Q, 16), np.uint8)
        check(lib().fec_relay_session_hop1_headers(h, self.hop1_hdr.ctypes.data_as(ctypes.c_void_p)),
              "fec_relay_session_hop1_headers")
        self.proc = np.zeros(Q, np.uint8)
        self.flag = np.zeros(Q, np.uint8)
        check(lib().fec_relay_session_dest_meta(h, self.proc.ctypes.data_as(ctypes.c_void_p),
                                                self.flag.ctypes.data_as(ctypes.c_void_p)), "fec_relay_session_dest_meta")

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                lib().fec_relay_session_destroy(self._h)
            except Exception:
                pass
            self._h = None

    def run(self, payload, relay=None, out=None, lost=None, count=None):
        """payload [Q, L] uint8 on the GPU -> (relay packets [relay_bytes] (packet t at
        relay_off[t]..relay_off[t+1]), destination outputs [Q, 320], lost flags [Q], lost count [1])."""
        import torch
        assert payload.dtype == torch.uint8 and payload.is_cuda and payload.is_contiguous()
        assert tuple(payload.shape) == (self.Q, self.L)
        dev = payload.device
        if relay is None:
            relay = torch.empty(int(self.relay_off[-1]), dtype=torch.uint8, device=dev)
        if out is None:
            out = torch.empty((self.Q, self.DW), dtype=torch.uint8, device=dev)
        if lost is None:
            lost = torch.empty(self.Q, dtype=torch.uint8, device=dev)
        if count is None:
            count = torch.empty(1, dtype=torch.int64, device=dev)
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        check(lib().fec_relay_session_run(self._h, _ptr(payload), _ptr(relay), _ptr(out), _ptr(lost), _ptr(count),
                                          stream), "fec_relay_session_run")
        return relay, out, lost, count

    def hop1_packets(self, stride: int):
        """After run(): the source's wire packets [Q, stride] (16-byte header + VR frame, zero padded)
        and their sizes [Q]."""
        import torch
        pk = torch.empty((self.Q, stride), dtype=torch.uint8, device="cuda")
        ln = torch.empty(self.Q, dtype=torch.int32, device="cuda")
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        check(lib().fec_relay_session_hop1(self._h, _ptr(pk), stride, _ptr(ln), stream), "fec_relay_session_hop1")
        return pk, ln


def relay_digest(frames, frame_len, out, flags, block: int = 100):
    """Per block of ``block`` seqs the CRC-32 of every seq's [frame_len LE32][frame][out][flag]
    (as tests/cpp/relay_dropin_test.cpp --digest writes for the reference-structured driver)."""
    import zlib
    import numpy as np
    fr = frames.cpu().numpy()
    fl = frame_len.cpu().numpy().astype(np.int64)
    ou = out.cpu().numpy()
    P = fr.shape[0]
    res = []
    for b0 in range(0, P, block):
        c = 0
        for t in range(b0, min(P, b0 + block)):
            c = zlib.crc32(int(fl[t]).to_bytes(4, "little"), c)
            c = zlib.crc32(fr[t, :fl[t]].tobytes(), c)
            c = zlib.crc32(ou[t].tobytes(), c)
            c = zlib.crc32(bytes([int(flags[t])]), c)
        res.append(c)
    return res
