"""Host-side mirror of the reference's coding API over the MI355X C ABI.

Two faces, both backed only by ``libfec_amd.so`` (no CPU fallback):

* ``FEC_Encoder`` / ``FEC_Decoder`` -- the reference's per-packet interface
  (src/FEC_Encoder.cpp:42-68 ``onTransmit``, src/FEC_Decoder.cpp:49-72 ``onReceive``): same
  constructor arguments, one call per sequence number from 0, same return meaning.
* ``Codec`` -- batched, device-resident encode/decode of a whole stream window held in HBM as
  torch uint8 tensors; launches on the current torch stream (torch is plumbing here: device
  memory and streams).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import KERNEL_NAMES, check, lib


def _stream_handle(torch):
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _check_out(torch, out, out_len, rows: int, width: int, device):
    """Allocate, or validate caller-supplied, output buffers of at least [rows, width] uint8 and
    [rows] int32 (the C side writes that many rows through raw pointers)."""
    if out is None:
        out = torch.empty((rows, width), dtype=torch.uint8, device=device)
    else:
        assert out.dtype == torch.uint8 and out.is_cuda and out.is_contiguous(), "out: contiguous uint8 GPU tensor"
        assert out.dim() == 2 and out.shape[1] == width and out.shape[0] >= rows, \
            f"out must be at least [{rows}, {width}], got {tuple(out.shape)}"
    if out_len is None:
        out_len = torch.empty(rows, dtype=torch.int32, device=device)
    else:
        assert out_len.dtype == torch.int32 and out_len.is_cuda and out_len.is_contiguous(), \
            "out_len: contiguous int32 GPU tensor"
        assert out_len.numel() >= rows, f"out_len must hold at least {rows} entries"
    return out, out_len


def _check_erasure(torch, erasure, P: int):
    assert erasure.dtype == torch.uint8 and erasure.is_cuda and erasure.is_contiguous(), \
        "erasure: contiguous uint8 GPU tensor"
    assert erasure.numel() >= P, f"erasure must hold at least {P} flags"


class Codec:
    """One (max_payload, T, B, N) configuration on the current HIP device.

    Geometry follows src/Encoder.cpp:31-39: k = T-N+1, n = k+B, S = ceil((max_payload+2)/k)
    sub-streams, CW = S*n untrimmed codeword bytes.
    """

    def __init__(self, max_payload: int, T: int, B: int, N: int):
        h = ctypes.c_void_p()
        check(lib().fec_codec_create(max_payload, T, B, N, ctypes.byref(h)), "fec_codec_create")
        self._h = h
        v = [ctypes.c_int() for _ in range(4)]
        check(lib().fec_codec_geometry(h, *[ctypes.byref(x) for x in v]), "fec_codec_geometry")
        self.k, self.n, self.S, self.CW = (x.value for x in v)
        self.L, self.T, self.B, self.N = max_payload, T, B, N
        self._ws = None

    def __del__(self):
        if getattr(self, "_h", None) and lib is not None:
            try:
                lib().fec_codec_destroy(self._h)
            except Exception:
                pass
            self._h = None

    # -- configuration ------------------------------------------------------------------------
    def generator(self) -> np.ndarray:
        """Encoder::getG() -- the k x n systematic generator matrix."""
        G = np.zeros(self.k * self.n, dtype=np.uint8)
        check(lib().fec_codec_generator(self._h, G.ctypes.data_as(ctypes.c_void_p)), "generator")
        return G.reshape(self.k, self.n)

    def set_encode_path(self, path: str) -> None:
        """'auto', 'generic' (fec_encode_kernel, any geometry and alignment) or 'tile' (the
        (k, n-k)-specialised LDS-tile kernel, auto's choice when it applies)."""
        code = {"auto": 0, "generic": 1, "tile": 5}[path]
        check(lib().fec_codec_set_encode_path(self._h, code), "fec_codec_set_encode_path")

    def set_copy_path(self, path: str) -> None:
        """'auto', 'generic' (fec_copy_kernel) or 'fast' (the (k, n-k)-specialised LDS-tile kernel,
        auto's choice when it applies) for the decoder's received-packet kernel."""
        code = {"auto": 0, "generic": 1, "fast": 2}[path]
        check(lib().fec_codec_set_copy_path(self._h, code), "fec_codec_set_copy_path")

    def info(self) -> dict:
        """Kernel configuration chosen for this codec on this device."""
        import json
        buf = ctypes.create_string_buffer(512)
        check(lib().fec_codec_info(self._h, buf, 512), "fec_codec_info")
        return json.loads(buf.value.decode())

    def set_plan_path(self, path: str) -> None:
        """'auto', 'generic' or 'fast' for the decoder's planner."""
        code = {"auto": 0, "generic": 1, "fast": 2}[path]
        check(lib().fec_codec_set_plan_path(self._h, code), "fec_codec_set_plan_path")

    def set_episode_dedup(self, on: bool) -> None:
        """Planner replays one episode per distinct loss shape (default) or every episode."""
        check(lib().fec_codec_set_episode_dedup(self._h, int(bool(on))), "fec_codec_set_episode_dedup")

    # -- block mode (relay): many independent code blocks ----------------------------------------
    def encode_blocks(self, data, out=None):
        """encodeBlock(t = k-1) per block (src/codingOperations.cpp:131-147): data [nblk, k] uint8 on
        the GPU -> codewords [nblk, n] = [data, parity]."""
        import torch
        assert data.dtype == torch.uint8 and data.is_cuda and data.dim() == 2 and data.shape[1] == self.k
        data = data.contiguous()
        if out is None:
            out = torch.empty((data.shape[0], self.n), dtype=torch.uint8, device=data.device)
        check(lib().fec_block_encode_batch(self._h, _ptr(data), data.shape[0], _ptr(out), _stream_handle(torch)),
              "fec_block_encode_batch")
        return out

    def decode_blocks(self, cw, erasure):
        """decodeBlock(T = n-1, t = 0) per block (src/codingOperations.cpp:149-232): codewords and
        erasure flags [nblk, n] uint8 on the GPU -> (codewords with the recovered data symbols
        written in, updated erasure flags)."""
        import torch
        assert cw.dtype == torch.uint8 and cw.is_cuda and cw.dim() == 2 and cw.shape[1] == self.n
        assert erasure.dtype == torch.uint8 and erasure.shape == cw.shape
        cw, erasure = cw.contiguous(), erasure.contiguous()
        out = torch.empty_like(cw)
        er_out = torch.empty_like(erasure)
        check(lib().fec_block_decode_batch(self._h, _ptr(cw), _ptr(erasure), cw.shape[0], _ptr(out), _ptr(er_out),
                                           _stream_handle(torch)), "fec_block_decode_batch")
        return out, er_out

    # -- batched device-resident path -----------------------------------------------------------
    def encode(self, payload, lengths=None, history: int = 0, out=None, out_len=None):
        """Encode rows ``history..`` of ``payload`` ([rows, L] uint8 on the GPU).

        Rows ``0..history-1`` are earlier packets of the same stream (context only).  Returns
        (codewords [P, CW] uint8, trimmed wire sizes [P] int32).
        """
        import torch
        assert payload.dtype == torch.uint8 and payload.is_cuda and payload.dim() == 2
        assert payload.shape[1] == self.L and payload.is_contiguous()
        P = payload.shape[0] - history
        assert 0 <= history <= payload.shape[0]
        if lengths is not None:
            assert lengths.dtype == torch.int32 and lengths.is_cuda and lengths.numel() == payload.shape[0]
            assert lengths.is_contiguous()
        out, out_len = _check_out(torch, out, out_len, P, self.CW, payload.device)
        row0 = payload[history:] if P > 0 else payload
        len0 = lengths[history:] if lengths is not None else None
        check(lib().fec_encode_batch(self._h, _ptr(row0), _ptr(len0), history, P, _ptr(out),
                                     _ptr(out_len), _stream_handle(torch)), "fec_encode_batch")
        return out, out_len

    def workspace(self, P: int):
        import torch
        nbytes = int(lib().fec_decode_workspace_bytes(self._h, P))
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        return self._ws

    def decode(self, codewords, erasure, out=None, out_len=None):
        """A fresh decoder fed packets 0..P-1: returns (payload [P-T, L], lengths [P-T])."""
        import torch
        assert codewords.dtype == torch.uint8 and codewords.is_cuda and codewords.is_contiguous()
        assert codewords.shape[1] == self.CW
        P = codewords.shape[0]
        _check_erasure(torch, erasure, P)
        Pout = max(0, P - self.T)
        out, out_len = _check_out(torch, out, out_len, Pout, self.L, codewords.device)
        ws = self.workspace(P)
        check(lib().fec_decode_batch(self._h, _ptr(codewords), _ptr(erasure), P, _ptr(out),
                                     _ptr(out_len), _ptr(ws), ws.numel(), _stream_handle(torch)),
              "fec_decode_batch")
        return out, out_len

    def plan(self, erasure, P: int | None = None):
        """Erasure-only half of the decode (scan + per-episode replay) on the current stream."""
        import torch
        P = erasure.numel() if P is None else P
        _check_erasure(torch, erasure, P)
        ws = self.workspace(P)
        check(lib().fec_decode_plan(self._h, _ptr(erasure), P, _ptr(ws), ws.numel(),
                                    _stream_handle(torch)), "fec_decode_plan")

    def apply(self, codewords, erasure, out=None, out_len=None):
        """Byte half of the decode (systematic copy + recovery); ordered after plan()."""
        import torch
        P = codewords.shape[0]
        assert codewords.dtype == torch.uint8 and codewords.is_cuda
        assert codewords.shape[1] == self.CW and codewords.is_contiguous()
        _check_erasure(torch, erasure, P)
        Pout = max(0, P - self.T)
        out, out_len = _check_out(torch, out, out_len, Pout, self.L, codewords.device)
        ws = self.workspace(P)
        check(lib().fec_decode_apply(self._h, _ptr(codewords), _ptr(erasure), P, _ptr(out),
                                     _ptr(out_len), _ptr(ws), ws.numel(), _stream_handle(torch)),
              "fec_decode_apply")
        return out, out_len

    def copy(self, codewords, erasure, out=None, out_len=None):
        """Received packets' rows and lengths (independent of plan()); erased packets' rows are
        written by recover()."""
        import torch
        P = codewords.shape[0]
        assert codewords.dtype == torch.uint8 and codewords.is_cuda
        assert codewords.shape[1] == self.CW and codewords.is_contiguous()
        _check_erasure(torch, erasure, P)
        Pout = max(0, P - self.T)
        out, out_len = _check_out(torch, out, out_len, Pout, self.L, codewords.device)
        check(lib().fec_decode_copy(self._h, _ptr(codewords), _ptr(erasure), P, _ptr(out),
                                    _ptr(out_len), _stream_handle(torch)), "fec_decode_copy")
        return out, out_len

    def recover(self, codewords, out, out_len):
        """Erased packets' rows and lengths: recovered bytes, or zeros and length 0 (after plan())."""
        import torch
        P = codewords.shape[0]
        assert codewords.dtype == torch.uint8 and codewords.is_cuda and codewords.is_contiguous()
        assert codewords.shape[1] == self.CW
        _check_out(torch, out, out_len, max(0, P - self.T), self.L, codewords.device)
        ws = self.workspace(P)
        check(lib().fec_decode_recover(self._h, _ptr(codewords), P, _ptr(out), _ptr(out_len),
                                       _ptr(ws), ws.numel(), _stream_handle(torch)),
              "fec_decode_recover")
        return out, out_len

    def plan_stats(self):
        """(replayed, filled) episodes of the last plan (synchronises the device)."""
        v = [ctypes.c_int64() for _ in range(2)]
        check(lib().fec_decode_plan_stats(_ptr(self._ws), *[ctypes.byref(x) for x in v]),
              "fec_decode_plan_stats")
        return tuple(int(x.value) for x in v)

    def counters(self):
        """(episodes, recovered, lost) of the last decode (synchronises the device)."""
        v = [ctypes.c_int64() for _ in range(3)]
        check(lib().fec_decode_counters(_ptr(self._ws), *[ctypes.byref(x) for x in v]),
              "fec_decode_counters")
        return tuple(x.value for x in v)

    # -- per-kernel HIP-event timing ----------------------------------------------------------
    def timing(self, enable: bool = True):
        check(lib().fec_timing_enable(self._h, int(enable)), "fec_timing_enable")

    def collect_timing(self):
        """{kernel name: (total ms, launches)} since the last collect (synchronises)."""
        n = len(KERNEL_NAMES)
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_int64 * n)()
        check(lib().fec_timing_collect(self._h, ms, cnt), "fec_timing_collect")
        return {KERNEL_NAMES[i]: (ms[i], cnt[i]) for i in range(n)}


class DecodeStream:
    """One stream decoded in consecutive batches (fec_decode_stream_push): the decoder state of
    src/Decoder.cpp:72-175 carries over from call to call, so the rows returned by successive
    push() calls, concatenated, equal Codec.decode over the whole stream."""

    def __init__(self, codec: Codec):
        self.codec = codec
        h = ctypes.c_void_p()
        check(lib().fec_decode_stream_create(ctypes.byref(h)), "fec_decode_stream_create")
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().fec_decode_stream_destroy(h)
            self._h = None

    def state(self) -> tuple[int, int]:
        """(packets pushed so far, packet the last push restarted the decode at)."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        check(lib().fec_decode_stream_state(self._h, ctypes.byref(a), ctypes.byref(b)), "fec_decode_stream_state")
        return a.value, b.value

    def push(self, codewords, erasure, erasure_host, history: int = 0, out=None, out_len=None):
        """codewords [history + P, CW], erasure [history + P] (GPU) and erasure_host (numpy, the
        same flags): the last P rows are the new packets, the first `history` rows the stream's
        packets in front of them.  Returns (payload [n, L], lengths [n]) for the packets whose
        output became available (all but the last T pushed)."""
        import torch
        c = self.codec
        assert codewords.dtype == torch.uint8 and codewords.is_cuda and codewords.is_contiguous()
        assert codewords.shape[1] == c.CW
        rows = codewords.shape[0]
        P = rows - history
        assert 0 <= history <= rows
        _check_erasure(torch, erasure, rows)
        eh = np.ascontiguousarray(erasure_host, dtype=np.uint8)
        assert eh.size >= rows
        out, out_len = _check_out(torch, out, out_len, max(P, 1), c.L, codewords.device)
        ws = c.workspace(rows)
        n = ctypes.c_int64()
        cw0 = ctypes.c_void_p(codewords.data_ptr() + history * c.CW)
        er0 = ctypes.c_void_p(erasure.data_ptr() + history)
        eh0 = ctypes.c_void_p(eh.ctypes.data + history)
        check(lib().fec_decode_stream_push(c._h, self._h, cw0, er0, eh0, P, history, _ptr(out), _ptr(out_len),
                                           ctypes.byref(n), _ptr(ws), ws.numel(), _stream_handle(torch)),
              "fec_decode_stream_push")
        return out[:n.value], out_len[:n.value]


class StreamGroup:
    """Many independent streams of one (T,B,N) (fec_streams_*): each call codes the next packet
    of every listed stream in one launch -- one FEC_Encoder and one FEC_Decoder per stream, held
    on the device."""

    def __init__(self, max_payload: int, T: int, B: int, N: int, nstreams: int):
        h = ctypes.c_void_p()
        check(lib().fec_streams_create(max_payload, T, B, N, nstreams, ctypes.byref(h)), "fec_streams_create")
        self._h = h
        self.L, self.T, self.nstreams = max_payload, T, nstreams
        # the geometry of Encoder.cpp:31-45 (k = T-N+1, n = k+B, S = ceil((L+2)/k), CW = S*n);
        # fec_streams_create has validated (T,B,N) against it
        self.k = T - N + 1
        self.n = self.k + B
        self.S = -(-(max_payload + 2) // self.k)
        self.CW = self.S * self.n

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().fec_streams_destroy(h)
            self._h = None

    def encode(self, ids, payload, lengths=None, out=None, out_len=None):
        """ids: host int32 [M] distinct stream ids; payload [M, L] uint8 GPU -> (cw [M, CW], sizes [M])."""
        import torch
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        M = ids.size
        assert payload.dtype == torch.uint8 and payload.is_cuda and payload.is_contiguous()
        assert tuple(payload.shape) == (M, self.L)
        if lengths is not None:
            assert lengths.dtype == torch.int32 and lengths.is_cuda and lengths.numel() == M
        out, out_len = _check_out(torch, out, out_len, M, self.CW, payload.device)
        check(lib().fec_streams_encode(self._h, ids.ctypes.data_as(ctypes.c_void_p), M, _ptr(payload), _ptr(lengths),
                                       _ptr(out), _ptr(out_len), _stream_handle(torch)), "fec_streams_encode")
        return out, out_len

    def decode(self, ids, erasure, codewords, out=None, out_len=None):
        """ids: host int32 [M]; erasure: host uint8 [M]; codewords [M, CW] GPU -> (payload [M, L],
        lengths [M]): row m = packet seq-T of stream ids[m]."""
        import torch
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        er = np.ascontiguousarray(erasure, dtype=np.uint8)
        M = ids.size
        assert er.size == M
        assert codewords.dtype == torch.uint8 and codewords.is_cuda and codewords.is_contiguous()
        assert tuple(codewords.shape) == (M, self.CW)
        out, out_len = _check_out(torch, out, out_len, M, self.L, codewords.device)
        check(lib().fec_streams_decode(self._h, ids.ctypes.data_as(ctypes.c_void_p), M,
                                       er.ctypes.data_as(ctypes.c_void_p), _ptr(codewords), _ptr(out), _ptr(out_len),
                                       _stream_handle(torch)), "fec_streams_decode")
        return out, out_len


class FEC_Encoder:
    """FEC_Encoder(max_payload, T, B, N) -- per-packet interface (src/FEC_Encoder.cpp:22-68)."""

    def __init__(self, max_payload: int, T: int, B: int, N: int, memory=None):
        h = ctypes.c_void_p()
        check(lib().fec_encoder_create(max_payload, T, B, N, ctypes.byref(h)), "FEC_Encoder")
        self._h = h
        self.T, self.B, self.N, self.max_payload = T, B, N, max_payload
        self.k = T - N + 1
        self.n = self.k + B
        self.max_blocklength = -(-(max_payload + 2) // self.k) * self.n
        self._cw = np.zeros(self.max_blocklength, dtype=np.uint8)

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                lib().fec_encoder_destroy(self._h)
            except Exception:
                pass
            self._h = None

    def onTransmit(self, data, payload: int, seq: int):
        """Returns (wire codeword bytes (trimmed), codeword_size)."""
        d = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data, dtype=np.uint8)
        if not 0 <= payload <= d.size:
            raise ValueError(f"payload {payload} exceeds the {d.size} data bytes given")
        size = ctypes.c_int()
        check(lib().fec_encoder_transmit(self._h, d.ctypes.data_as(ctypes.c_void_p), payload, seq,
                                         self._cw.ctypes.data_as(ctypes.c_void_p), ctypes.byref(size)),
              "onTransmit")
        return self._cw[:size.value].copy(), size.value


class FEC_Decoder:
    """FEC_Decoder(max_payload, T, B, N) -- per-packet interface (src/FEC_Decoder.cpp:26-72)."""

    def __init__(self, max_payload: int, T: int, B: int, N: int, memory=None):
        h = ctypes.c_void_p()
        check(lib().fec_decoder_create(max_payload, T, B, N, ctypes.byref(h)), "FEC_Decoder")
        self._h = h
        self.T, self.B, self.N, self.max_payload = T, B, N, max_payload
        self._out = np.zeros(max_payload, dtype=np.uint8)

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                lib().fec_decoder_destroy(self._h)
            except Exception:
                pass
            self._h = None

    def onReceive(self, codeword, codeword_size: int, seq: int, erasure: bool):
        """Returns (payload bytes of packet seq-T (max_payload, zero past the payload), payload)."""
        p = ctypes.c_int()
        if erasure or codeword is None:
            st = lib().fec_decoder_receive(self._h, None, 0, seq, 1,
                                           self._out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(p))
        else:
            c = np.ascontiguousarray(codeword, dtype=np.uint8)
            if not 0 <= codeword_size <= c.size:
                raise ValueError(f"codeword_size {codeword_size} exceeds the {c.size} bytes given")
            st = lib().fec_decoder_receive(self._h, c.ctypes.data_as(ctypes.c_void_p), codeword_size,
                                           seq, 0, self._out.ctypes.data_as(ctypes.c_void_p),
                                           ctypes.byref(p))
        check(st, "onReceive")
        return self._out.copy(), p.value


def plan_host(max_payload: int, T: int, B: int, N: int, erasure: np.ndarray) -> np.ndarray:
    """Symbolic decoder on the host: fate of packets 0..P-T-1 (1 copy, 2 recovered, 3 lost)."""
    e = np.ascontiguousarray(erasure, dtype=np.uint8)
    fate = np.zeros(e.size, dtype=np.uint8)
    check(lib().fec_plan_host(max_payload, T, B, N, e.ctypes.data_as(ctypes.c_void_p), e.size,
                              fate.ctypes.data_as(ctypes.c_void_p)), "fec_plan_host")
    return fate[: max(0, e.size - T)]
