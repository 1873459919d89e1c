"""ctypes wrapper around the CPU oracle (oracle/ricepp_oracle.c).

TEST INFRASTRUCTURE ONLY: the parity checker and the CPU-baseline leg of
bench.py.  Never imported by the product package ``dwarfs_amd``.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "libricepp_oracle.so"

OK = 0
UNSUPPORTED_CONFIG = -1
TRUNCATED_INPUT = -2
INVALID_ARGUMENT = -3
OUTPUT_TOO_SMALL = -4


class Config(C.Structure):
    _fields_ = [
        ("block_size", C.c_uint32),
        ("component_stream_count", C.c_uint32),
        ("big_endian", C.c_uint32),
        ("unused_lsb_count", C.c_uint32),
    ]


def build() -> Path:
    if not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < (HERE / "ricepp_oracle.c").stat().st_mtime:
        subprocess.run(["make", "-C", str(HERE), "-s"], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(str(LIB_PATH))
        P = C.c_void_p
        L.rpo_check_config.argtypes = [C.POINTER(Config)]
        L.rpo_worst_case_bytes.argtypes = [C.POINTER(Config), C.c_size_t]
        L.rpo_worst_case_bytes.restype = C.c_size_t
        L.rpo_encode.argtypes = [C.POINTER(Config), P, C.c_size_t, P, C.c_size_t, C.POINTER(C.c_size_t)]
        L.rpo_decode.argtypes = [C.POINTER(Config), P, C.c_size_t, P, C.c_size_t]
        L.rpo_bitstream_run_ops.argtypes = [P, P, P, C.c_size_t, P, C.c_size_t, C.POINTER(C.c_long)]
        L.rpo_bitstream_run_ops.restype = C.c_long
        L.rpo_encode_batch.argtypes = [C.POINTER(Config), P, P, P, C.c_size_t, P, P, P, P, P, C.c_int]
        L.rpo_encode_batch.restype = None
        L.rpo_decode_batch.argtypes = [C.POINTER(Config), P, P, P, C.c_size_t, P, P, P, P, C.c_int]
        L.rpo_decode_batch.restype = None
        L.rpo_frame_header.argtypes = [P, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_uint32]
        L.rpo_frame_header.restype = C.c_size_t
        _lib = L
    return _lib


def cfg(block_size=128, cs=1, big_endian=True, ulsb=0) -> Config:
    return Config(block_size, cs, 1 if big_endian else 0, ulsb)


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class OracleError(RuntimeError):
    def __init__(self, status: int):
        super().__init__(f"oracle status {status}")
        self.status = status


def worst_case_bytes(c: Config, n: int) -> int:
    return lib().rpo_worst_case_bytes(C.byref(c), n)


def encode(c: Config, samples: np.ndarray) -> bytes:
    samples = np.ascontiguousarray(samples, dtype=np.uint16)
    st = lib().rpo_check_config(C.byref(c))
    if st:
        raise OracleError(st)
    cap = worst_case_bytes(c, samples.size)
    out = np.zeros(max(cap, 1), np.uint8)
    n = C.c_size_t(0)
    st = lib().rpo_encode(C.byref(c), _p(samples), samples.size, _p(out), cap, C.byref(n))
    if st:
        raise OracleError(st)
    return out[: n.value].tobytes()


def decode(c: Config, data: bytes, n_samples: int) -> np.ndarray:
    buf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
    out = np.zeros(max(n_samples, 1), np.uint16)
    st = lib().rpo_decode(C.byref(c), _p(buf), len(data), _p(out), n_samples)
    if st:
        raise OracleError(st)
    return out[:n_samples]


def bitstream_run_ops(ops, bits, values):
    ops = np.asarray(ops, np.uint8)
    bits = np.asarray(bits, np.uint32)
    values = np.asarray(values, np.uint64)
    cap = int(bits.sum() // 8 + len(ops) + 64)
    out = np.zeros(cap, np.uint8)
    bad = C.c_long(0)
    n = lib().rpo_bitstream_run_ops(_p(ops), _p(bits), _p(values), len(ops), _p(out), cap, C.byref(bad))
    return out[:n].tobytes(), bad.value


def encode_batch(c: Config, samples: np.ndarray, in_off, n_samples, out_cap_each, nthreads=1):
    """Encodes independent blocks; returns (out buffer, out offsets, sizes, status)."""
    in_off = np.asarray(in_off, np.uint64)
    n_samples = np.asarray(n_samples, np.uint64)
    nb = len(in_off)
    caps = np.asarray(out_cap_each, np.uint64) if np.ndim(out_cap_each) else np.full(nb, out_cap_each, np.uint64)
    out_off = np.zeros(nb, np.uint64)
    if nb:
        out_off[1:] = np.cumsum(caps)[:-1]
    out = np.zeros(int(caps.sum()) + 1, np.uint8)
    sizes = np.zeros(nb, np.uint64)
    status = np.zeros(nb, np.int32)
    lib().rpo_encode_batch(C.byref(c), _p(samples), _p(in_off), _p(n_samples), nb, _p(out), _p(out_off),
                           _p(caps), _p(sizes), _p(status), nthreads)
    return out, out_off, sizes, status


def decode_batch(c: Config, data: np.ndarray, in_off, in_bytes, out_off, n_samples, total_samples, nthreads=1):
    in_off = np.asarray(in_off, np.uint64)
    in_bytes = np.asarray(in_bytes, np.uint64)
    out_off = np.asarray(out_off, np.uint64)
    n_samples = np.asarray(n_samples, np.uint64)
    out = np.zeros(max(total_samples, 1), np.uint16)
    status = np.zeros(len(in_off), np.int32)
    lib().rpo_decode_batch(C.byref(c), _p(data), _p(in_off), _p(in_bytes), len(in_off), _p(out), _p(out_off),
                           _p(n_samples), _p(status), nthreads)
    return out, status


def frame_header(uncompressed_bytes, block_size, component_count, bytes_per_sample, ulsb, big_endian, version=1):
    out = np.zeros(64, np.uint8)
    n = lib().rpo_frame_header(_p(out), uncompressed_bytes, block_size, component_count, bytes_per_sample, ulsb,
                               1 if big_endian else 0, version)
    return out[:n].tobytes()


def unused_lsb_count(samples: np.ndarray, big_endian: bool = True) -> int:
    """get_unused_lsb_count<uint16_t> (src/writer/categorizer/fits_categorizer.cpp:
    118-178): std::countr_zero of the OR of all samples (after the big-endian
    conversion of :161), 16 for an all-zero or empty image."""
    a = np.asarray(samples, dtype=np.uint16)
    b16 = int(np.bitwise_or.reduce(a)) if a.size else 0
    if big_endian:
        b16 = ((b16 >> 8) | (b16 << 8)) & 0xFFFF
    if b16 == 0:
        return 16
    return (b16 & -b16).bit_length() - 1


def _pcm_args(big_endian, is_signed, lsb_padded, nbytes, bits):
    if not 1 <= nbytes <= 4:
        # src/pcm_sample_transformer.cpp:310-311
        raise RuntimeError(f"unsupported number of bytes per sample: {nbytes}")
    if not 1 <= bits <= 8 * nbytes:  # asserted at :354
        raise ValueError(f"bits {bits} outside 1..{8 * nbytes}")


def pcm_unpack(packed, big_endian, is_signed, lsb_padded, nbytes, bits) -> np.ndarray:
    """pcm_sample_transformer<int32_t>::unpack (src/pcm_sample_transformer.cpp:
    50-93 byte assembly, :141-158 unpack_native), vectorised over samples with
    uint32 arithmetic mod 2^32: Lsb padding shifts right by 8*bytes-bits;
    signed sign-extends from bit bits-1 when bits < 32 (upper bits otherwise
    kept, no masking); unsigned subtracts 1 << (bits-1)."""
    _pcm_args(big_endian, is_signed, lsb_padded, nbytes, bits)
    b = np.frombuffer(bytes(packed), np.uint8).reshape(-1, nbytes).astype(np.uint32)
    t = np.zeros(b.shape[0], np.uint32)
    for k in range(nbytes):
        sh = 8 * (nbytes - 1 - k) if big_endian else 8 * k
        t |= b[:, k] << np.uint32(sh)
    if lsb_padded:
        t >>= np.uint32(8 * nbytes - bits)
    if is_signed:
        if bits < 32:
            neg = (t & np.uint32(1 << (bits - 1))) != 0
            t = np.where(neg, t | np.uint32((0xFFFFFFFF << bits) & 0xFFFFFFFF), t)
    else:
        t = t - np.uint32(1 << (bits - 1))
    return t.astype(np.uint32).view(np.int32)


def pcm_pack(samples, big_endian, is_signed, lsb_padded, nbytes, bits) -> bytes:
    """pcm_sample_transformer<int32_t>::pack (src/pcm_sample_transformer.cpp:
    160-171 pack_native, :97-138 byte order): unsigned adds 1 << (bits-1), Lsb
    padding shifts left by 8*bytes-bits, the low `bytes` bytes are stored."""
    _pcm_args(big_endian, is_signed, lsb_padded, nbytes, bits)
    s = np.asarray(samples, np.int32).view(np.uint32).copy()
    if not is_signed:
        s = s + np.uint32(1 << (bits - 1))
    if lsb_padded:
        s = s << np.uint32(8 * nbytes - bits)
    out = np.zeros((s.shape[0], nbytes), np.uint8)
    for k in range(nbytes):
        sh = 8 * (nbytes - 1 - k) if big_endian else 8 * k
        out[:, k] = (s >> np.uint32(sh)) & np.uint32(0xFF)
    return out.tobytes()
