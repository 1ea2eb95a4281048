"""Variable-rate (adaptive) coding -- BASELINE config 4 -- over the C ABI (fec_vr.cpp).

``VrPlan`` runs the reference's P2P loop (Application_Layer_Sender -> Variable_Rate_FEC_Encoder
-> erasure -> Application_Layer_Receiver with its Parameter_Estimator pair ->
Variable_Rate_FEC_Decoder, 6-byte feedback to the sender; application_local_simulation.cpp:328-345)
symbolically on the host: which (T,B,N) encodes each packet, where double coding starts and
stops, which decoder instance reports each packet and whether it is lost.  ``encode`` /
``decode`` then do the byte work of that schedule on the GPU, batched per coder instance.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib
from .codec import _ptr, _stream_handle


class VrPlan:
    def __init__(self, erasure: np.ndarray, P: int, max_payload: int = 300, T: int = 10, B: int = -1,
                 N: int = -1, adaptive_mode_MDS: bool = False, light: bool = False):
        """light=True: only the statistics are read back (the schedule arrays stay in the C plan,
        which is all encode()/decode() need)."""
        pat = np.ascontiguousarray(erasure, dtype=np.uint8)
        h = ctypes.c_void_p()
        check(lib().fec_vr_plan_create(max_payload, T, B, N, int(adaptive_mode_MDS),
                                       pat.ctypes.data_as(ctypes.c_void_p), pat.size, P, ctypes.byref(h)),
              "fec_vr_plan_create")
        self._h = h
        self.L, self.T, self.P = max_payload, T, P
        self._load(light)

    def rerun(self, erasure: np.ndarray, P: int, wait: bool = True, light: bool = True):
        """Plan again in place (same configuration) on another pattern / P, reusing the plan's
        buffers.  wait=False returns after the control loop: the symbolic decoders run on worker
        threads meanwhile (encode() can launch at once; decode() and the statistics wait for them)."""
        pat = np.ascontiguousarray(erasure, dtype=np.uint8)
        check(lib().fec_vr_plan_rerun(self._h, pat.ctypes.data_as(ctypes.c_void_p), pat.size, P, 0 if wait else 1),
              "fec_vr_plan_rerun")
        self.P = P
        if wait:
            self._load(light)
        else:
            sent, cwm = ctypes.c_int64(), ctypes.c_int()
            check(lib().fec_vr_plan_stats(self._h, None, None, None, ctypes.byref(sent), None, None, ctypes.byref(cwm)),
                  "fec_vr_plan_stats")
            self.sent, self.cw_max = sent.value, cwm.value
        return self

    def _load(self, light):
        h, P = self._h, self.P
        lost, sw, sent = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        rate = ctypes.c_double()
        ne, nd, cwm = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().fec_vr_plan_stats(h, ctypes.byref(lost), ctypes.byref(sw), ctypes.byref(rate),
                                      ctypes.byref(sent), ctypes.byref(ne), ctypes.byref(nd), ctypes.byref(cwm)),
              "fec_vr_plan_stats")
        self.lost, self.switches, self.coding_rate = lost.value, sw.value, rate.value
        self.sent, self.cw_max = sent.value, cwm.value
        c_ms, d_ms = ctypes.c_double(), ctypes.c_double()
        check(lib().fec_vr_plan_timing(h, ctypes.byref(c_ms), ctypes.byref(d_ms)), "fec_vr_plan_timing")
        fw = ctypes.c_double()
        lib().fec_vr_plan_feedback_wait.restype = ctypes.c_int
        check(lib().fec_vr_plan_feedback_wait(h, ctypes.byref(fw)), "fec_vr_plan_feedback_wait")
        self.plan_ms = {"control_loop": c_ms.value, "decoder_instances": d_ms.value, "feedback_wait": fw.value}
        if light:
            return
        self.encoders = np.zeros((ne.value, 6), dtype=np.int64)
        self.decoders = np.zeros((nd.value, 6), dtype=np.int64)
        check(lib().fec_vr_plan_instances(h, self.encoders.ctypes.data_as(ctypes.c_void_p),
                                          self.decoders.ctypes.data_as(ctypes.c_void_p)), "fec_vr_plan_instances")
        self.frames = np.zeros((self.sent, 6), dtype=np.int32)
        self.erased = np.zeros(self.sent, dtype=np.uint8)
        self.fate = np.zeros(P, dtype=np.uint8)
        self.fate_decoder = np.zeros(P, dtype=np.int32)
        check(lib().fec_vr_plan_packets(h, *(a.ctypes.data_as(ctypes.c_void_p) for a in
                                             (self.frames, self.erased, self.fate, self.fate_decoder))),
              "fec_vr_plan_packets")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().fec_vr_plan_destroy(h)
            self._h = None

    def tuples(self) -> set:
        return {tuple(int(v) for v in r[:3]) for r in self.encoders}

    # -- batched device-resident path -----------------------------------------------------------
    def layout(self):
        """(cur_bytes, old_bytes): sizes of the compact codeword arrays (fec_vr.h)."""
        cb, ob = ctypes.c_int64(), ctypes.c_int64()
        check(lib().fec_vr_plan_layout(self._h, ctypes.byref(cb), ctypes.byref(ob)), "fec_vr_plan_layout")
        return cb.value, ob.value

    def row_offsets(self):
        """(cur_off, old_off) int64 [sent+1] each: row s of the cur / old array spans
        [off[s], off[s+1]) (empty old rows for frames without double coding)."""
        co = np.zeros(self.sent + 1, dtype=np.int64)
        oo = np.zeros(self.sent + 1, dtype=np.int64)
        check(lib().fec_vr_plan_row_offsets(self._h, co.ctypes.data_as(ctypes.c_void_p),
                                            oo.ctypes.data_as(ctypes.c_void_p)), "fec_vr_plan_row_offsets")
        return co, oo

    @staticmethod
    def rows(arr, off, first: int, end: int, width: int):
        """Rows [first, end) of one encoder instance (consecutive at stride CW rounded to 16) of a
        compact array as a [end-first, width] view."""
        if end <= first:
            return arr[:0].view(0, width)
        o0 = int(off[first])
        stride = int(off[first + 1] - off[first])
        return arr[o0:o0 + (end - first) * stride].view(end - first, stride)[:, :width]

    def alloc_frames(self, device="cuda", zero=True):
        """(cw_cur, len_cur, cw_old, len_old) buffers for encode(): the two compact codeword arrays
        (1-D, fec_vr_plan_layout's sizes) and the per-frame trimmed sizes."""
        import torch
        mk = torch.zeros if zero else torch.empty
        cb, ob = self.layout()
        return (mk(max(cb, 16), dtype=torch.uint8, device=device),
                torch.zeros(self.sent, dtype=torch.int32, device=device),
                mk(max(ob, 16), dtype=torch.uint8, device=device),
                torch.zeros(self.sent, dtype=torch.int32, device=device))

    def encode(self, payload, lengths=None, frames=None):
        """payload: [sent, L] uint8 on the GPU -> (cw_cur, len_cur, cw_old, len_old): the codewords
        every frame carries in the compact arrays (row_offsets()), trimmed sizes (old: 0 if none)."""
        import torch
        assert payload.dtype == torch.uint8 and payload.is_cuda and tuple(payload.shape) == (self.sent, self.L)
        cw_cur, len_cur, cw_old, len_old = frames if frames is not None else self.alloc_frames(payload.device)
        check(lib().fec_vr_encode_batch(self._h, _ptr(payload), _ptr(lengths), _ptr(cw_cur), _ptr(len_cur),
                                        _ptr(cw_old), _ptr(len_old), _stream_handle(torch)), "fec_vr_encode_batch")
        return cw_cur, len_cur, cw_old, len_old

    def decode(self, cw_cur, cw_old, erased=None, out=None, out_len=None):
        """-> (payload out [P, L], lengths [P], 0 = lost): the receiver's reported outputs (every
        row is written)."""
        import torch
        dev = cw_cur.device
        if erased is None:  # the device decode does not read it (the plan holds the pattern)
            erased = out
        if out is None:
            out = torch.empty((self.P, self.L), dtype=torch.uint8, device=dev)
        if out_len is None:
            out_len = torch.empty(self.P, dtype=torch.int32, device=dev)
        check(lib().fec_vr_decode_batch(self._h, _ptr(cw_cur), _ptr(cw_old), _ptr(erased), _ptr(out), _ptr(out_len),
                                        _stream_handle(torch)), "fec_vr_decode_batch")
        return out, out_len

    # -- wire framing above the boundary ---------------------------------------------------------
    def wire_packets(self, cw_cur, len_cur, cw_old, len_old, packets=None, packet_len=None):
        """The P2P wire packets the sender emits (Application_Layer_Sender.cpp:259-269 +
        Variable_Rate_FEC_Encoder.cpp:194-217): rows [sent, 10 + 2*cw_max] uint8 and sizes [sent]."""
        import torch
        stride = 10 + 2 * self.cw_max
        dev = cw_cur.device
        if packets is None:
            packets = torch.zeros((self.sent, stride), dtype=torch.uint8, device=dev)
        if packet_len is None:
            packet_len = torch.empty(self.sent, dtype=torch.int32, device=dev)
        assert packets.shape == (self.sent, stride) and packets.is_contiguous() and packet_len.numel() >= self.sent
        check(lib().fec_vr_frames_batch(self._h, _ptr(cw_cur), _ptr(len_cur), _ptr(cw_old), _ptr(len_old),
                                        _ptr(packets), stride, _ptr(packet_len), _stream_handle(torch)),
              "fec_vr_frames_batch")
        return packets, packet_len


def parse_packets(plan: "VrPlan", packets, packet_len):
    """The receiver's split of the plan's P2P wire packets (rows [sent, stride] uint8 on the GPU)
    into the current / old codeword rows of the compact arrays (zero-padded to their row size) and
    header fields [sent, 5] (seq, T, B, N, counter)."""
    import torch
    assert packets.dtype == torch.uint8 and packets.is_cuda and packets.is_contiguous() and packets.dim() == 2
    R = packets.shape[0]
    assert R == plan.sent and packet_len.dtype == torch.int32 and packet_len.numel() >= R
    cb, ob = plan.layout()
    cur = torch.empty(max(cb, 16), dtype=torch.uint8, device=packets.device)
    old = torch.empty(max(ob, 16), dtype=torch.uint8, device=packets.device)
    hdr = torch.empty((R, 5), dtype=torch.int32, device=packets.device)
    check(lib().fec_vr_parse_batch(plan._h, _ptr(packets), packets.shape[1], _ptr(packet_len), _ptr(cur), _ptr(old),
                                   _ptr(hdr), _stream_handle(torch)), "fec_vr_parse_batch")
    return cur, old, hdr
