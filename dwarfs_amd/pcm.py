"""Host-side mirror of DwarFS's ``pcm_sample_transformer<int32_t>`` over the
MI355X kernels of ``dwarfs_amd/csrc/pcm_transform.hip``.

Mirrors include/dwarfs/pcm_sample_transformer.h:36-71: the three format enums,
the constructor ``(endianness, signedness, padding, bytes, bits)`` and
``unpack(dst, src)`` / ``pack(dst, src)`` over spans of the same sample count
(src/pcm_sample_transformer.cpp:44-228).  Here the spans are CUDA tensors
(``uint8`` packed bytes, ``int32`` samples) and the work is one launch of the
C ABI ``rpp_pcm_unpack`` / ``rpp_pcm_pack`` on the current stream.

Errors follow the reference: an unsupported byte count raises
``RuntimeError("unsupported number of bytes per sample: N")``
(src/pcm_sample_transformer.cpp:310-311); ``bits`` outside 1..8*bytes (an
assert in the reference, :354) raises ``ValueError``; mismatched spans (the
reference's asserts at :185,194) raise ``ValueError``.
"""

from __future__ import annotations

import ctypes as C
import enum
from typing import Optional

import torch

from . import _native as N

__all__ = [
    "PcmSampleEndianness",
    "PcmSampleSignedness",
    "PcmSamplePadding",
    "PcmSampleTransformer",
]


class PcmSampleEndianness(enum.Enum):
    Big = 0
    Little = 1

    def __str__(self) -> str:  # operator<< (src/pcm_sample_transformer.cpp:381-384)
        return "big-endian" if self is PcmSampleEndianness.Big else "little-endian"


class PcmSampleSignedness(enum.Enum):
    Signed = 0
    Unsigned = 1

    def __str__(self) -> str:  # :386-389
        return "signed" if self is PcmSampleSignedness.Signed else "unsigned"


class PcmSamplePadding(enum.Enum):
    Lsb = 0
    Msb = 1

    def __str__(self) -> str:  # :391-394
        return "lsb-padded" if self is PcmSamplePadding.Lsb else "msb-padded"


class PcmSampleTransformer:
    """``pcm_sample_transformer<int32_t>`` (pcm_sample_transformer.h:40-71)."""

    def __init__(self, end: PcmSampleEndianness, sig: PcmSampleSignedness, pad: PcmSamplePadding,
                 nbytes: int, bits: int):
        self.fmt = N.RppPcmFormat(
            1 if end is PcmSampleEndianness.Big else 0,
            1 if sig is PcmSampleSignedness.Signed else 0,
            1 if pad is PcmSamplePadding.Lsb else 0,
            int(nbytes) if 0 <= int(nbytes) < 2**32 else 0,
            int(bits) if 0 <= int(bits) < 2**32 else 0,
        )
        st = N.lib().rpp_pcm_check_format(C.byref(self.fmt))
        if st == N.RPP_UNSUPPORTED_CONFIG or not 1 <= int(nbytes) <= 4:
            raise RuntimeError(f"unsupported number of bytes per sample: {nbytes}")
        if st != N.RPP_OK:
            raise ValueError(f"bits {bits} outside 1..{8 * int(nbytes)}")
        self.bytes = int(nbytes)
        self.bits = int(bits)

    @staticmethod
    def _check_dev(t: torch.Tensor, dtype: torch.dtype, what: str) -> None:
        if not isinstance(t, torch.Tensor) or not t.is_cuda:
            raise ValueError(f"{what} must be a CUDA tensor")
        if t.dtype != dtype or not t.is_contiguous():
            raise ValueError(f"{what} must be a contiguous {dtype} tensor")

    def unpack(self, dst: torch.Tensor, src: torch.Tensor, stream: Optional[torch.cuda.Stream] = None) -> None:
        """dst (int32, n) <- src (uint8, bytes*n) -- ``unpack`` (:183-190)."""
        self._check_dev(dst, torch.int32, "dst")
        self._check_dev(src, torch.uint8, "src")
        if src.numel() != self.bytes * dst.numel():
            raise ValueError("unpack: src must hold bytes * dst.size() bytes")
        s = stream if stream is not None else torch.cuda.current_stream(dst.device)
        st = N.lib().rpp_pcm_unpack(C.byref(self.fmt), C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
                                    dst.numel(), C.c_void_p(s.cuda_stream))
        if st != N.RPP_OK:
            raise RuntimeError(f"rpp_pcm_unpack: {N.STATUS_NAMES.get(st, st)}")

    def pack(self, dst: torch.Tensor, src: torch.Tensor, stream: Optional[torch.cuda.Stream] = None) -> None:
        """dst (uint8, bytes*n) <- src (int32, n) -- ``pack`` (:192-199)."""
        self._check_dev(dst, torch.uint8, "dst")
        self._check_dev(src, torch.int32, "src")
        if dst.numel() != self.bytes * src.numel():
            raise ValueError("pack: dst must hold bytes * src.size() bytes")
        s = stream if stream is not None else torch.cuda.current_stream(src.device)
        st = N.lib().rpp_pcm_pack(C.byref(self.fmt), C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
                                  src.numel(), C.c_void_p(s.cuda_stream))
        if st != N.RPP_OK:
            raise RuntimeError(f"rpp_pcm_pack: {N.STATUS_NAMES.get(st, st)}")
