"""ctypes binding of the in-tree HIP library ``libfec_amd.so`` (C ABI: include/fec_amd.h).

The library is the product: there is no CPU fallback.  If it is missing the import of any op
fails loudly with instructions to build it (``python -c "import __graft_entry__ as g; g.build()"``
or ``make -C fec_erasure_code_unit_test_relay_amd/csrc``).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FEC_AMD_LIB: an A/B build of the same sources (csrc/Makefile OUT=..., e.g. another -D variant)
LIB_PATH = os.environ.get("FEC_AMD_LIB") or os.path.join(_HERE, "libfec_amd.so")
HEADER_PATHS = [os.path.join(_HERE, "..", "include", "fec_amd.h")]

FEC_OK = 0
FEC_ERR_ARG = -1
FEC_ERR_HIP = -2
FEC_ERR_NOMEM = -3
FEC_ERR_WORKSPACE = -4
FEC_ERR_SEQUENCE = -5
FEC_ERR_HISTORY = -6

KERNEL_NAMES = ["fec_encode_kernel", "fec_scan_kernel", "fec_plan_kernel", "fec_copy_kernel",
                "fec_recover_kernel"]


class FecError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        msg = lib().fec_strerror(status).decode() if _lib is not None else str(status)
        if status == FEC_ERR_HIP and _lib is not None:  # which HIP call failed, and where
            buf = ctypes.create_string_buffer(512)
            if _lib.fec_last_error(buf, len(buf)) > 0:
                msg += f" [{buf.value.decode(errors='replace')}]"
        super().__init__(f"{what}: {msg} (status {status})")
        self.status = status


_lib = None


def lib() -> ctypes.CDLL:
    """Load libfec_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: the HIP extension must be built first "
            "(make -C fec_erasure_code_unit_test_relay_amd/csrc); there is no fallback")
    # torch ships its own libamdhip64.so.7 (same SONAME as /opt/rocm's): whichever is loaded first
    # serves the whole process.  Load torch's first so that the tensors torch allocates and the
    # kernels this library launches share one HIP runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    ip = ctypes.POINTER(ctypes.c_int)
    i64p = ctypes.POINTER(ctypes.c_int64)
    L.fec_strerror.restype = ctypes.c_char_p
    L.fec_strerror.argtypes = [i32]
    L.fec_last_error.restype = i32
    L.fec_last_error.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    L.fec_version.restype = i32
    L.fec_codec_create.argtypes = [i32, i32, i32, i32, ctypes.POINTER(vp)]
    L.fec_codec_destroy.argtypes = [vp]
    L.fec_codec_geometry.argtypes = [vp, ip, ip, ip, ip]
    L.fec_codec_generator.argtypes = [vp, vp]
    L.fec_codec_set_encode_path.argtypes = [vp, i32]
    L.fec_codec_set_copy_path.argtypes = [vp, i32]
    L.fec_codec_set_plan_path.argtypes = [vp, i32]
    L.fec_codec_info.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t]
    L.fec_codec_set_episode_dedup.argtypes = [vp, i32]
    L.fec_debug_stamps.argtypes = [vp, i32, vp]
    L.fec_encode_batch.argtypes = [vp, vp, vp, i64, i64, vp, vp, vp]
    L.fec_decode_workspace_bytes.restype = ctypes.c_size_t
    L.fec_decode_workspace_bytes.argtypes = [vp, i64]
    L.fec_decode_batch.argtypes = [vp, vp, vp, i64, vp, vp, vp, ctypes.c_size_t, vp]
    L.fec_decode_counters.argtypes = [vp, i64p, i64p, i64p]
    L.fec_streams_create.argtypes = [i32, i32, i32, i32, i32, ctypes.POINTER(vp)]
    L.fec_streams_destroy.argtypes = [vp]
    L.fec_streams_encode.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp]
    L.fec_streams_decode.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp]
    L.fec_streams_state.argtypes = [vp, i32, i64p, i64p]
    L.fec_decode_stream_create.argtypes = [ctypes.POINTER(vp)]
    L.fec_decode_stream_destroy.argtypes = [vp]
    L.fec_decode_stream_state.argtypes = [vp, i64p, i64p]
    L.fec_decode_stream_push.argtypes = [vp, vp, vp, vp, vp, i64, i64, vp, vp, i64p, vp, ctypes.c_size_t, vp]
    L.fec_decode_plan_stats.argtypes = [vp, i64p, i64p]
    L.fec_decode_plan.argtypes = [vp, vp, i64, vp, ctypes.c_size_t, vp]
    L.fec_decode_apply.argtypes = [vp, vp, vp, i64, vp, vp, vp, ctypes.c_size_t, vp]
    L.fec_decode_copy.argtypes = [vp, vp, vp, i64, vp, vp, vp]
    L.fec_decode_recover.argtypes = [vp, vp, i64, vp, vp, vp, ctypes.c_size_t, vp]
    L.fec_timing_enable.argtypes = [vp, i32]
    L.fec_timing_collect.argtypes = [vp, ctypes.POINTER(ctypes.c_double), i64p]
    L.fec_encoder_create.argtypes = [i32, i32, i32, i32, ctypes.POINTER(vp)]
    L.fec_encoder_destroy.argtypes = [vp]
    L.fec_encoder_transmit.argtypes = [vp, vp, i32, i32, vp, ip]
    L.fec_decoder_create.argtypes = [i32, i32, i32, i32, ctypes.POINTER(vp)]
    L.fec_decoder_destroy.argtypes = [vp]
    L.fec_decoder_receive.argtypes = [vp, vp, i32, i32, i32, vp, ip]
    L.fec_plan_host.argtypes = [i32, i32, i32, i32, vp, i64, vp]
    L.fec_util_fill_payload.argtypes = [vp, i64, i64, i32, ctypes.c_uint64, vp]
    f32 = ctypes.c_float
    L.fec_erasure_iid.argtypes = [vp, i32, f32, i32]
    L.fec_erasure_three_sections_iid.argtypes = [vp, i32, f32, i32, f32, i32, f32, i32]
    L.fec_erasure_ge.argtypes = [vp, i32, f32, f32, f32, i32, ip]
    L.fec_erasure_ge_varying.argtypes = [vp, i32, f32, f32, f32, i32, ip]
    L.fec_erasure_fritchman_varying.argtypes = [vp, i32, f32, f32, f32, i32, i32]
    L.fec_erasure_periodic.argtypes = [vp, i32, i32, i32, i32]
    L.fec_block_encode_batch.argtypes = [vp, vp, i64, vp, vp]
    L.fec_block_decode_batch.argtypes = [vp, vp, vp, i64, vp, vp, vp]
    L.fec_vr_plan_create.argtypes = [i32, i32, i32, i32, i32, vp, i64, i64, ctypes.POINTER(vp)]
    L.fec_vr_plan_destroy.argtypes = [vp]
    L.fec_vr_plan_rerun.argtypes = [vp, vp, i64, i64, i32]
    L.fec_vr_plan_stats.argtypes = [vp, i64p, i64p, ctypes.POINTER(ctypes.c_double), i64p, ip, ip, ip]
    L.fec_vr_plan_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    L.fec_vr_plan_instances.argtypes = [vp, vp, vp]
    L.fec_vr_plan_packets.argtypes = [vp, vp, vp, vp, vp]
    L.fec_vr_encode_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp]
    L.fec_vr_decode_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    L.fec_vr_frames_batch.argtypes = [vp, vp, vp, vp, vp, vp, i64, vp, vp]
    L.fec_vr_parse_batch.argtypes = [vp, vp, i64, vp, vp, vp, vp, vp]
    L.fec_vr_plan_layout.argtypes = [vp, i64p, i64p]
    L.fec_vr_plan_row_offsets.argtypes = [vp, vp, vp]
    L.fec_swdf_create.argtypes = [i32, i32, i32, i32, i32, ctypes.POINTER(vp)]
    L.fec_swdf_destroy.argtypes = [vp]
    L.fec_swdf_geometry.argtypes = [vp, ip, ip, ip, ip, ip, ip]
    L.fec_swdf_workspace_bytes.restype = ctypes.c_size_t
    L.fec_swdf_workspace_bytes.argtypes = [vp, i64]
    L.fec_swdf_relay_batch.argtypes = [vp, vp, i64, vp, i64, vp, vp, vp, ctypes.c_size_t, vp]
    L.fec_swdf_destination_batch.argtypes = [vp, vp, vp, i64, vp, vp, vp]
    L.fec_sdswdf_create.argtypes = [i32, i32, i32, i32, i32, i32, ctypes.POINTER(vp)]
    L.fec_sdswdf_destroy.argtypes = [vp]
    L.fec_sdswdf_geometry.argtypes = [vp, ip, ip, ip, ip, ip, ip, ip]
    L.fec_sdswdf_tile_geometry.argtypes = [i32, i32, i32, i32, i32, i32, i64, ip, ip]
    L.fec_sdswdf_relay_batch.argtypes = [vp, vp, i64, vp, i64, vp, vp]
    L.fec_sdswdf_destination_batch.argtypes = [vp, vp, vp, i64, vp, vp, vp]
    L.fec_sdswdf_relay_plan.argtypes = [vp, vp, i64, vp, vp, i64, i64p, ip]
    L.fec_sdswdf_dest_plan.argtypes = [vp, vp, vp, i64, vp, vp, vp, i64, i64p, ip]
    L.fec_sdswdf_relay_batch_starts.argtypes = [vp, vp, i64, vp, i64, vp, i32, vp, vp]
    L.fec_sdswdf_destination_batch_starts.argtypes = [vp, vp, vp, i64, vp, i32, vp, vp, vp]
    L.fec_relay_vr_create.argtypes = [i32, i32, vp, i32, i64, ctypes.POINTER(vp)]
    L.fec_relay_vr_destroy.argtypes = [vp]
    L.fec_relay_vr_geometry.argtypes = [vp, ip, ip, ip]
    L.fec_relay_vr_run.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.fec_relay_session_create.argtypes = [i32, i32, i64, vp, i64, vp, i64, ctypes.POINTER(vp)]
    L.fec_relay_session_destroy.argtypes = [vp]
    L.fec_relay_session_info.argtypes = [vp, vp, vp]
    L.fec_relay_session_relay_offsets.argtypes = [vp, vp]
    L.fec_relay_session_hop1_headers.argtypes = [vp, vp]
    L.fec_relay_session_dest_meta.argtypes = [vp, vp, vp]
    L.fec_relay_session_run.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    L.fec_relay_session_hop1.argtypes = [vp, vp, i64, vp, vp]
    for name in ["fec_relay_session_create", "fec_relay_session_destroy", "fec_relay_session_info",
                 "fec_relay_session_relay_offsets", "fec_relay_session_hop1_headers", "fec_relay_session_dest_meta",
                 "fec_relay_session_run", "fec_relay_session_hop1", "fec_sdswdf_create", "fec_sdswdf_destroy", "fec_sdswdf_geometry", "fec_sdswdf_tile_geometry", "fec_sdswdf_relay_batch",
                 "fec_sdswdf_destination_batch", "fec_sdswdf_relay_plan", "fec_sdswdf_dest_plan",
                 "fec_sdswdf_relay_batch_starts", "fec_sdswdf_destination_batch_starts", "fec_relay_vr_create",
                 "fec_relay_vr_destroy", "fec_relay_vr_geometry", "fec_relay_vr_run",
                 "fec_swdf_create", "fec_swdf_destroy", "fec_swdf_geometry", "fec_swdf_relay_batch",
                 "fec_swdf_destination_batch", "fec_codec_create", "fec_codec_destroy", "fec_codec_set_encode_path",
                 "fec_codec_set_copy_path", "fec_codec_set_plan_path", "fec_codec_info", "fec_codec_set_episode_dedup", "fec_debug_stamps", "fec_codec_geometry",
                 "fec_codec_generator", "fec_encode_batch", "fec_decode_batch", "fec_decode_plan",
                 "fec_decode_stream_create", "fec_decode_stream_destroy", "fec_decode_stream_state",
                 "fec_decode_stream_push", "fec_streams_create", "fec_streams_destroy", "fec_streams_encode",
                 "fec_streams_decode", "fec_streams_state",
                 "fec_decode_apply", "fec_decode_copy", "fec_decode_recover",
                 "fec_decode_counters", "fec_decode_plan_stats", "fec_timing_enable", "fec_timing_collect",
                 "fec_encoder_create", "fec_encoder_destroy", "fec_encoder_transmit",
                 "fec_decoder_create", "fec_decoder_destroy", "fec_decoder_receive",
                 "fec_plan_host", "fec_util_fill_payload", "fec_erasure_iid",
                 "fec_erasure_three_sections_iid", "fec_erasure_ge", "fec_erasure_ge_varying",
                 "fec_erasure_fritchman_varying", "fec_erasure_periodic", "fec_vr_plan_create",
                 "fec_vr_plan_rerun", "fec_vr_plan_destroy", "fec_vr_plan_stats", "fec_vr_plan_timing", "fec_vr_plan_instances", "fec_vr_plan_packets",
                 "fec_vr_encode_batch", "fec_vr_decode_batch", "fec_vr_frames_batch", "fec_vr_parse_batch",
                 "fec_vr_plan_layout", "fec_vr_plan_row_offsets", "fec_block_encode_batch",
                 "fec_block_decode_batch"]:
        getattr(L, name).restype = i32
    _lib = L
    return _lib


def check(status: int, what: str) -> None:
    if status != FEC_OK:
        raise FecError(status, what)
