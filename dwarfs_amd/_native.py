"""Loader for the native MI355X ricepp library (libricepp_amd.so).

The library exports exactly the C ABI of ``include/ricepp_amd.h``.  There is
no fallback: if the library is missing or fails to load, every entry point
raises, so a GPU run can never silently pass on a non-native path.
"""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("RICEPP_AMD_LIB", PKG / "lib" / "libricepp_amd.so"))

RPP_OK = 0
RPP_UNSUPPORTED_CONFIG = -1
RPP_TRUNCATED_INPUT = -2
RPP_INVALID_ARGUMENT = -3
RPP_OUTPUT_TOO_SMALL = -4
RPP_HIP_ERROR = -5
RPP_INTERNAL_ERROR = -6

RPP_DECODE_AUTO = 0
RPP_DECODE_FUSED = 1
RPP_DECODE_SEGMENTED = 2
RPP_TEST_NO_FAST_LANES = 1
RPP_TEST_LOOKBACK_STALL = 2
RPP_TEST_PHASE_TIMERS = 4

STATUS_NAMES = {
    RPP_OK: "OK",
    RPP_UNSUPPORTED_CONFIG: "UNSUPPORTED_CONFIG",
    RPP_TRUNCATED_INPUT: "TRUNCATED_INPUT",
    RPP_INVALID_ARGUMENT: "INVALID_ARGUMENT",
    RPP_OUTPUT_TOO_SMALL: "OUTPUT_TOO_SMALL",
    RPP_HIP_ERROR: "HIP_ERROR",
    RPP_INTERNAL_ERROR: "INTERNAL_ERROR",
}

# Every symbol declared in include/ricepp_amd.h.
EXPORTED_SYMBOLS = (
    "rpp_abi_version",
    "rpp_check_config",
    "rpp_worst_case_bytes",
    "rpp_encode_batch",
    "rpp_encode_workspace_bytes",
    "rpp_encode_batch_ws",
    "rpp_decode_batch",
    "rpp_decode_workspace_bytes",
    "rpp_decode_batch_ws",
    "rpp_decode_workspace_bytes_ex",
    "rpp_decode_batch_ex",
    "rpp_unused_lsb_batch",
    "rpp_exclusive_scan_u64",
    "rpp_pack_batch",
    "rpp_frame_header",
    "rpp_parse_frame",
    "rpp_pcm_check_format",
    "rpp_pcm_unpack",
    "rpp_pcm_pack",
    "rpp_flac_frame_header",
    "rpp_flac_parse_frame",
    "rpp_flac_stream_header",
    "rpp_flac_parse_stream",
    "rpp_flac_frame_bound",
    "rpp_flac_encode_workspace_bytes",
    "rpp_flac_encode",
    "rpp_flac_encode_ex",
    "rpp_flac_encode_batch_workspace_bytes",
    "rpp_flac_encode_batch",
    "rpp_flac_decode_workspace_bytes",
    "rpp_flac_decode",
    "rpp_flac_decode_batch_workspace_bytes",
    "rpp_flac_decode_batch",
)


class RppConfig(C.Structure):
    """``rpp_config`` (mirrors ricepp::codec_config, codec_config.h:36-41)."""

    _fields_ = [
        ("block_size", C.c_uint32),
        ("component_stream_count", C.c_uint32),
        ("big_endian", C.c_uint32),
        ("unused_lsb_count", C.c_uint32),
    ]


class RppDecodeOptions(C.Structure):
    """``rpp_decode_options`` (explicit decode path selection, tests and diagnostics)."""

    _fields_ = [
        ("path", C.c_uint32),
        ("seg_log2", C.c_uint32),
        ("fused_waves", C.c_uint32),
        ("test_flags", C.c_uint32),
    ]


class RppFrame(C.Structure):
    _fields_ = [
        ("uncompressed_bytes", C.c_uint64),
        ("block_size", C.c_uint32),
        ("component_count", C.c_uint32),
        ("bytes_per_sample", C.c_uint32),
        ("unused_lsb_count", C.c_uint32),
        ("big_endian", C.c_uint32),
        ("ricepp_version", C.c_uint32),
    ]


class RppFlacFrame(C.Structure):
    """``rpp_flac_frame`` (the flac_block_header fields, thrift/compression.thrift:36-40)."""

    _fields_ = [
        ("uncompressed_bytes", C.c_uint64),
        ("num_channels", C.c_uint32),
        ("bits_per_sample", C.c_uint32),
        ("flags", C.c_uint32),
    ]


class RppFlacStreamInfo(C.Structure):
    _fields_ = [
        ("min_blocksize", C.c_uint32),
        ("max_blocksize", C.c_uint32),
        ("sample_rate", C.c_uint32),
        ("channels", C.c_uint32),
        ("bits_per_sample", C.c_uint32),
        ("total_samples", C.c_uint64),
    ]


class RppPcmFormat(C.Structure):
    """``rpp_pcm_format`` (pcm_sample_transformer's constructor arguments,
    include/dwarfs/pcm_sample_transformer.h:36-45)."""

    _fields_ = [
        ("big_endian", C.c_uint32),
        ("is_signed", C.c_uint32),
        ("lsb_padded", C.c_uint32),
        ("bytes", C.c_uint32),
        ("bits", C.c_uint32),
    ]


_lib = None


def lib() -> C.CDLL:
    """Returns the loaded native library; raises if it is not built."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"native ricepp library not found at {LIB_PATH}; run `python __graft_entry__.py build`"
            )
        L = C.CDLL(str(LIB_PATH))
        P = C.c_void_p
        L.rpp_abi_version.restype = C.c_uint32
        L.rpp_check_config.argtypes = [C.POINTER(RppConfig)]
        L.rpp_check_config.restype = C.c_int
        L.rpp_worst_case_bytes.argtypes = [C.POINTER(RppConfig), C.c_uint64]
        L.rpp_worst_case_bytes.restype = C.c_uint64
        L.rpp_encode_batch.argtypes = [C.POINTER(RppConfig), P, P, P, C.c_uint32, P, P, P, P, P]
        L.rpp_encode_batch.restype = C.c_int
        L.rpp_encode_workspace_bytes.argtypes = [C.POINTER(RppConfig), C.c_uint64, C.c_uint64, C.c_uint32]
        L.rpp_encode_workspace_bytes.restype = C.c_uint64
        L.rpp_encode_batch_ws.argtypes = [C.POINTER(RppConfig), P, P, P, C.c_uint32, P, P, P, P, C.c_uint64,
                                          C.c_uint64, P, C.c_uint64, P]
        L.rpp_encode_batch_ws.restype = C.c_int
        L.rpp_decode_batch.argtypes = [C.POINTER(RppConfig), P, P, P, C.c_uint32, P, P, P, P, P]
        L.rpp_decode_batch.restype = C.c_int
        L.rpp_decode_workspace_bytes.argtypes = [C.POINTER(RppConfig), C.c_uint64, C.c_uint64, C.c_uint32]
        L.rpp_decode_workspace_bytes.restype = C.c_uint64
        L.rpp_decode_batch_ws.argtypes = [C.POINTER(RppConfig), P, P, P, C.c_uint32, P, P, P, P, C.c_uint64,
                                          C.c_uint64, P, C.c_uint64, P]
        L.rpp_decode_batch_ws.restype = C.c_int
        L.rpp_decode_workspace_bytes_ex.argtypes = [C.POINTER(RppConfig), C.c_uint64, C.c_uint64, C.c_uint32,
                                                    C.POINTER(RppDecodeOptions)]
        L.rpp_decode_workspace_bytes_ex.restype = C.c_uint64
        L.rpp_decode_batch_ex.argtypes = [C.POINTER(RppConfig), P, P, P, C.c_uint32, P, P, P, P, C.c_uint64,
                                          C.c_uint64, P, C.c_uint64, C.POINTER(RppDecodeOptions), P]
        L.rpp_decode_batch_ex.restype = C.c_int
        L.rpp_unused_lsb_batch.argtypes = [P, P, P, C.c_uint64, C.c_uint32, C.c_uint32, P, P, P]
        L.rpp_unused_lsb_batch.restype = C.c_int
        L.rpp_exclusive_scan_u64.argtypes = [P, C.c_uint64, P, P]
        L.rpp_exclusive_scan_u64.restype = C.c_int
        L.rpp_pack_batch.argtypes = [P, P, P, C.c_uint32, P, P, P, P]
        L.rpp_pack_batch.restype = C.c_int
        L.rpp_frame_header.argtypes = [C.POINTER(RppFrame), P]
        L.rpp_frame_header.restype = C.c_size_t
        L.rpp_parse_frame.argtypes = [P, C.c_size_t, C.POINTER(RppFrame)]
        L.rpp_parse_frame.restype = C.c_long
        L.rpp_pcm_check_format.argtypes = [C.POINTER(RppPcmFormat)]
        L.rpp_pcm_check_format.restype = C.c_int
        L.rpp_pcm_unpack.argtypes = [C.POINTER(RppPcmFormat), P, P, C.c_uint64, P]
        L.rpp_pcm_unpack.restype = C.c_int
        L.rpp_pcm_pack.argtypes = [C.POINTER(RppPcmFormat), P, P, C.c_uint64, P]
        L.rpp_pcm_pack.restype = C.c_int
        L.rpp_flac_frame_header.argtypes = [C.POINTER(RppFlacFrame), P]
        L.rpp_flac_frame_header.restype = C.c_size_t
        L.rpp_flac_parse_frame.argtypes = [P, C.c_size_t, C.POINTER(RppFlacFrame)]
        L.rpp_flac_parse_frame.restype = C.c_long
        L.rpp_flac_stream_header.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64, P]
        L.rpp_flac_stream_header.restype = C.c_size_t
        L.rpp_flac_parse_stream.argtypes = [P, C.c_size_t, C.POINTER(RppFlacStreamInfo)]
        L.rpp_flac_parse_stream.restype = C.c_long
        L.rpp_flac_frame_bound.argtypes = [C.c_uint32, C.c_uint32]
        L.rpp_flac_frame_bound.restype = C.c_uint64
        L.rpp_flac_encode_workspace_bytes.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32]
        L.rpp_flac_encode_workspace_bytes.restype = C.c_uint64
        L.rpp_flac_encode.argtypes = [P, C.c_uint64, C.c_uint32, C.c_uint32, P, P, P, C.c_uint64, P]
        L.rpp_flac_encode.restype = C.c_int
        L.rpp_flac_encode_ex.argtypes = [P, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P, P, P,
                                         C.c_uint64, P]
        L.rpp_flac_encode_ex.restype = C.c_int
        L.rpp_flac_encode_batch_workspace_bytes.argtypes = [C.c_uint32, P, P, P]
        L.rpp_flac_encode_batch_workspace_bytes.restype = C.c_uint64
        L.rpp_flac_encode_batch.argtypes = [P, C.c_uint32, P, P, P, P, C.c_uint32, C.c_uint32, P, P, P, C.c_uint64, P]
        L.rpp_flac_encode_batch.restype = C.c_int
        L.rpp_flac_decode_workspace_bytes.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
        L.rpp_flac_decode_workspace_bytes.restype = C.c_uint64
        L.rpp_flac_decode.argtypes = [P, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, P, P,
                                      C.c_uint32, P, C.c_uint64, P, P]
        L.rpp_flac_decode.restype = C.c_int
        L.rpp_flac_decode_batch_workspace_bytes.argtypes = [C.c_uint32, P, P, P, P, P]
        L.rpp_flac_decode_batch_workspace_bytes.restype = C.c_uint64
        L.rpp_flac_decode_batch.argtypes = [P, C.c_uint32, P, P, P, P, P, P, P, P, P, P, P, C.c_uint64, P, P]
        L.rpp_flac_decode_batch.restype = C.c_int
        if L.rpp_abi_version() != 1:
            raise RuntimeError("libricepp_amd.so ABI mismatch")
        _lib = L
    return _lib
