"""Host-side mirror of the ricepp library API over the MI355X kernels.

Mirrors ``ricepp::create_encoder<uint16_t>`` / ``create_decoder<uint16_t>``
(ricepp/include/ricepp/create_encoder.h:39-41, create_decoder.h:39-41) and the
``encoder_interface`` / ``decoder_interface`` methods
(ricepp/include/ricepp/encoder_interface.h:38-60, decoder_interface.h:37-50),
plus batched device-resident entry points that are the MI355X-native way to
drive the codec: many independent blocks per launch, one wavefront per block.

Error behaviour follows the reference:
  * invalid config  -> ``RuntimeError("Unsupported configuration")``
    (ricepp/ricepp_cpuspecific.cpp:161,173)
  * reading past the end of the input -> ``OutOfRange`` (an ``IndexError``,
    the Python analogue of ``std::out_of_range``, bitstream_reader.h:150-152)

Everything here calls the C ABI of ``include/ricepp_amd.h``; there is no CPU
codec in this package.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence, Union

import numpy as np
import torch

from . import _native as N

__all__ = [
    "CodecConfig",
    "OutOfRange",
    "UnsupportedConfiguration",
    "Encoder",
    "Decoder",
    "EncodedBatch",
    "create_encoder",
    "create_decoder",
    "worst_case_encoded_bytes",
    "encode_batch",
    "decode_batch",
    "DecodeOptions",
]


class UnsupportedConfiguration(RuntimeError):
    """``std::runtime_error("Unsupported configuration")``."""

    def __init__(self) -> None:
        super().__init__("Unsupported configuration")


class OutOfRange(IndexError):
    """``std::out_of_range``: the decoder ran past the end of its input."""


class CodecError(RuntimeError):
    pass


@dataclass(frozen=True)
class CodecConfig:
    """``ricepp::codec_config`` (ricepp/include/ricepp/codec_config.h:36-41)."""

    block_size: int = 128
    component_stream_count: int = 1
    byteorder: str = "big"  # "big" or "little": byte order of the stored samples
    unused_lsb_count: int = 0

    def native(self) -> N.RppConfig:
        if self.byteorder not in ("big", "little"):
            raise ValueError(f"byteorder must be 'big' or 'little', not {self.byteorder!r}")
        return N.RppConfig(
            int(self.block_size),
            int(self.component_stream_count),
            1 if self.byteorder == "big" else 0,
            int(self.unused_lsb_count),
        )


def _raise_status(st: int) -> None:
    if st == N.RPP_OK:
        return
    if st == N.RPP_UNSUPPORTED_CONFIG:
        raise UnsupportedConfiguration()
    if st == N.RPP_TRUNCATED_INPUT:
        raise OutOfRange("bitstream_reader::read_packet")
    raise CodecError(f"ricepp_amd: {N.STATUS_NAMES.get(st, st)}")


def _check(config: CodecConfig) -> N.RppConfig:
    c = config.native()
    _raise_status(N.lib().rpp_check_config(C.byref(c)))
    return c


def worst_case_encoded_bytes(config: CodecConfig, n_samples: int) -> int:
    c = _check(config)
    return int(N.lib().rpp_worst_case_bytes(C.byref(c), int(n_samples)))


def _stream_ptr(stream: Optional[torch.cuda.Stream]) -> C.c_void_p:
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def _dev_u64(values, device) -> torch.Tensor:
    return torch.as_tensor(np.asarray(values, dtype=np.int64), device=device)


def _dev_u64_many(device, *arrays):
    """Several host int64 arrays in one host-to-device copy (a small batch's call is latency-bound: one copy
    instead of one per array); returns device views, one per array (a device tensor passes through)."""
    host = [a for a in arrays if not isinstance(a, torch.Tensor)]
    flat = np.concatenate([np.asarray(a, dtype=np.int64).reshape(-1) for a in host]) if host else np.zeros(0, np.int64)
    d = torch.as_tensor(flat, device=device)
    out, at = [], 0
    for a in arrays:
        if isinstance(a, torch.Tensor):
            out.append(a)
            continue
        n = np.asarray(a).size
        out.append(d[at:at + n])
        at += n
    return out


def _as_u16_tensor(samples, device) -> torch.Tensor:
    if isinstance(samples, torch.Tensor):
        if samples.element_size() != 2:
            raise TypeError("samples must be a 16-bit tensor")
        t = samples.reshape(-1)
        if t.device.type != "cuda":
            t = t.to(device)
        return t.contiguous()
    a = np.ascontiguousarray(np.asarray(samples), dtype=np.uint16)
    return torch.from_numpy(a.view(np.int16)).to(device)


@dataclass
class EncodedBatch:
    """Device-resident result of :func:`encode_batch`."""

    data: torch.Tensor          # uint8 [sum of per-block capacities]
    offsets: np.ndarray         # int64 [nblocks] byte offset of each block's stream (host)
    d_offsets: torch.Tensor     # same, on the device
    sizes: torch.Tensor         # int64 [nblocks] encoded bytes (device)
    status: torch.Tensor        # int32 [nblocks] (device)

    def check(self) -> None:
        st = self.status.cpu().numpy()
        bad = np.nonzero(st)[0]
        if len(bad):
            _raise_status(int(st[bad[0]]))

    def block(self, i: int) -> bytes:
        n = int(self.sizes[i].item())
        o = int(self.offsets[i])
        return self.data[o:o + n].cpu().numpy().tobytes()


def encode_batch(
    config: CodecConfig,
    samples: torch.Tensor,
    in_offsets: Sequence[int],
    n_samples: Sequence[int],
    stream: Optional[torch.cuda.Stream] = None,
    out: Optional[torch.Tensor] = None,
    out_offsets: Optional[np.ndarray] = None,
) -> EncodedBatch:
    """Encodes independent blocks of device-resident samples in one launch.

    ``samples`` is a 16-bit CUDA tensor of *stored* samples (the byte order
    named by ``config.byteorder``); block ``b`` is
    ``samples[in_offsets[b] : in_offsets[b] + n_samples[b]]``.
    """
    c = _check(config)
    dev = samples.device
    n_samples = np.asarray(n_samples, dtype=np.int64)
    nb = len(n_samples)
    if out_offsets is None:
        # (one rpp_worst_case_bytes call per distinct length)
        uniq, inv = np.unique(n_samples, return_inverse=True)
        caps = np.array([N.lib().rpp_worst_case_bytes(C.byref(c), int(n)) for n in uniq], np.int64)[inv]
        caps = (caps + 15) // 16 * 16
        out_offsets = np.zeros(nb, np.int64)
        if nb:
            out_offsets[1:] = np.cumsum(caps)[:-1]
        total = int(caps.sum()) if nb else 0
    else:
        total = None
    if out is None:
        out = torch.empty(max(total or 0, 16), dtype=torch.uint8, device=dev)
    d_in_off, d_n, d_out_off = _dev_u64_many(dev, in_offsets, n_samples, out_offsets)
    sizes = torch.empty(nb, dtype=torch.int64, device=dev)
    status = torch.empty(nb, dtype=torch.int32, device=dev)
    total_samples = int(n_samples.sum()) if nb else 0
    max_samples = int(n_samples.max()) if nb else 0
    ws = encode_workspace(config, total_samples, max_samples, nb, dev, stream)
    st = N.lib().rpp_encode_batch_ws(
        C.byref(c), C.c_void_p(samples.data_ptr()), C.c_void_p(d_in_off.data_ptr()),
        C.c_void_p(d_n.data_ptr()), nb, C.c_void_p(out.data_ptr()), C.c_void_p(d_out_off.data_ptr()),
        C.c_void_p(sizes.data_ptr()), C.c_void_p(status.data_ptr()), total_samples, max_samples,
        C.c_void_p(ws.data_ptr()), ws.numel(), _stream_ptr(stream))
    _raise_status(st)
    return EncodedBatch(out, np.asarray(out_offsets, np.int64), d_out_off, sizes, status)


def encode_workspace(config: CodecConfig, total_samples: int, max_stream_samples: int, nblocks: int, device,
                     stream=None) -> torch.Tensor:
    """Device workspace of ``rpp_encode_batch_ws`` (segment table and scratch for streams encoded by
    several waves) for ``nblocks`` streams of ``total_samples`` samples, none longer than
    ``max_stream_samples``."""
    c = _check(config)
    nbytes = int(N.lib().rpp_encode_workspace_bytes(C.byref(c), int(total_samples), int(max_stream_samples),
                                                    int(nblocks)))
    ws = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
    if stream is not None:
        ws.record_stream(stream)
    return ws


_PATHS = {"auto": N.RPP_DECODE_AUTO, "fused": N.RPP_DECODE_FUSED, "segmented": N.RPP_DECODE_SEGMENTED}


@dataclass(frozen=True)
class DecodeOptions:
    """``rpp_decode_options``: explicit decode path selection (tests, diagnostics, tuning).  The default is
    exactly ``rpp_decode_batch_ws``: segmented when the batch has long streams, else one wave per stream."""

    path: str = "auto"        # "auto", "fused" (one wave per stream) or "segmented" (split every long stream)
    seg_log2: int = 0         # units of 2**seg_log2 bits (10..26); 0: chosen from the batch
    fused_waves: int = 0      # streams per workgroup of the fused kernel (1..16); 0: auto
    test_flags: int = 0       # RPP_TEST_* fault injection / diagnostics

    def native(self) -> N.RppDecodeOptions:
        if self.path not in _PATHS:
            raise ValueError(f"decode path must be one of {sorted(_PATHS)}, not {self.path!r}")
        return N.RppDecodeOptions(_PATHS[self.path], int(self.seg_log2), int(self.fused_waves), int(self.test_flags))


def decode_batch(
    config: CodecConfig,
    data: torch.Tensor,
    in_offsets: Sequence[int],
    in_bytes: Union[Sequence[int], torch.Tensor],
    n_samples: Sequence[int],
    stream: Optional[torch.cuda.Stream] = None,
    out: Optional[torch.Tensor] = None,
    out_offsets: Optional[Sequence[int]] = None,
    options: Optional[DecodeOptions] = None,
):
    """Decodes independent blocks of a device-resident encoded buffer.

    Returns ``(samples int16 tensor, status int32 tensor)``.  Block ``b``'s
    samples land at ``out[out_offsets[b] : out_offsets[b] + n_samples[b]]``
    (default: packed back to back).
    """
    c = _check(config)
    dev = data.device
    n_samples = np.asarray(n_samples, dtype=np.int64)
    nb = len(n_samples)
    if out_offsets is None:
        out_offsets = np.zeros(nb, np.int64)
        if nb:
            out_offsets[1:] = np.cumsum(n_samples)[:-1]
    out_offsets = np.asarray(out_offsets, np.int64)
    if out is None:
        total = int((out_offsets + n_samples).max()) if nb else 0
        out = torch.empty(max(total, 8), dtype=torch.int16, device=dev)
    d_in_off, d_in_bytes, d_n, d_out_off = _dev_u64_many(dev, in_offsets, in_bytes, n_samples, out_offsets)
    status = torch.empty(nb, dtype=torch.int32, device=dev)
    total = int(n_samples.sum()) if nb else 0
    longest = int(n_samples.max()) if nb else 0
    ws = decode_workspace(config, total, nb, dev, longest, options)
    if stream is not None:
        ws.record_stream(stream)
    o = (options or DecodeOptions()).native()
    st = N.lib().rpp_decode_batch_ex(
        C.byref(c), C.c_void_p(data.data_ptr()), C.c_void_p(d_in_off.data_ptr()),
        C.c_void_p(d_in_bytes.data_ptr()), nb, C.c_void_p(out.data_ptr()), C.c_void_p(d_out_off.data_ptr()),
        C.c_void_p(d_n.data_ptr()), C.c_void_p(status.data_ptr()), total, longest, C.c_void_p(ws.data_ptr()),
        ws.numel(), C.byref(o), _stream_ptr(stream))
    _raise_status(st)
    return out, status


def segmented_decode_stats(reset: bool = True) -> dict:
    """Counters of the segmented decode since the last reset (diagnostics): units whose guessed chain met
    the exact one at once, reruns from a known header, serial passes, streams left to the fused kernel, and
    failed units that had found no guess at all."""
    buf = (C.c_ulonglong * 8)()
    _raise_status(N.lib().rpp_seg_diag_read(buf, int(reset)))
    return dict(zip(("met", "reruns", "serial", "fallback", "no_guess"), map(int, buf)))


def decode_workspace(config: CodecConfig, total_samples: int, nblocks: int, device,
                     max_stream_samples: Optional[int] = None, options: Optional[DecodeOptions] = None) -> torch.Tensor:
    """Device workspace of ``rpp_decode_batch_ws`` for a batch of ``nblocks`` streams of ``total_samples``
    samples, the longest ``max_stream_samples`` (default: ``total_samples``, i.e. sized for the segmented
    decode of long streams whenever the batch could need it)."""
    c = _check(config)
    mx = int(total_samples if max_stream_samples is None else max_stream_samples)
    o = (options or DecodeOptions()).native()
    nbytes = int(N.lib().rpp_decode_workspace_bytes_ex(C.byref(c), int(total_samples), mx, int(nblocks), C.byref(o)))
    return torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)


def unused_lsb_count_batch(
    samples: torch.Tensor,
    offsets: Sequence[int],
    n_samples: Sequence[int],
    big_endian: bool = True,
    stream: Optional[torch.cuda.Stream] = None,
) -> torch.Tensor:
    """Unused least-significant bits of 16-bit images, one launch per batch.

    The FITS categorizer's ``get_unused_lsb_count<uint16_t>``
    (src/writer/categorizer/fits_categorizer.cpp:118-178): the number of
    trailing zero bits of the OR of all samples of an image (16 for an
    all-zero or empty image).  Image ``i`` is
    ``samples[offsets[i] : offsets[i] + n_samples[i]]``.  Returns an int32
    device tensor of counts.
    """
    dev = samples.device
    n_samples = np.asarray(n_samples, dtype=np.int64)
    ni = len(n_samples)
    counts = torch.empty(ni, dtype=torch.int32, device=dev)
    if ni == 0:
        return counts
    d_off = _dev_u64(offsets, dev)
    d_n = _dev_u64(n_samples, dev)
    work = torch.empty(ni, dtype=torch.int32, device=dev)
    # the C ABI takes at most 65535 images per call (grid.y): slices
    for i0 in range(0, ni, _LSB_MAX_IMAGES):
        i1 = min(ni, i0 + _LSB_MAX_IMAGES)
        st = N.lib().rpp_unused_lsb_batch(
            C.c_void_p(samples.data_ptr()), C.c_void_p(d_off.data_ptr() + 8 * i0),
            C.c_void_p(d_n.data_ptr() + 8 * i0), int(n_samples[i0:i1].max()), i1 - i0, 1 if big_endian else 0,
            C.c_void_p(work.data_ptr() + 4 * i0), C.c_void_p(counts.data_ptr() + 4 * i0), _stream_ptr(stream))
        _raise_status(st)
    return counts


_LSB_MAX_IMAGES = 65535


class Encoder:
    """``encoder_interface<uint16_t>`` (encoder_interface.h:38-60)."""

    def __init__(self, config: CodecConfig, device: Union[str, torch.device] = "cuda"):
        _check(config)
        self.config = config
        self.device = torch.device(device)

    def worst_case_encoded_bytes(self, n_or_samples) -> int:
        n = n_or_samples if isinstance(n_or_samples, (int, np.integer)) else len(n_or_samples)
        return worst_case_encoded_bytes(self.config, int(n))

    def encode(self, samples) -> bytes:
        """``encode(span<u16 const>) -> vector<u8>`` (ricepp_cpuspecific.cpp:53-56,91-99)."""
        t = _as_u16_tensor(samples, self.device)
        res = encode_batch(self.config, t, [0], [t.numel()])
        res.check()
        return res.block(0)

    def encode_into(self, out: np.ndarray, samples) -> int:
        """``encode(span<u8>, span<u16 const>) -> span<u8>``: returns the bytes used."""
        data = self.encode(samples)
        if len(out) < self.worst_case_encoded_bytes(samples):
            raise ValueError("output buffer smaller than worst_case_encoded_bytes")
        out[: len(data)] = np.frombuffer(data, np.uint8)
        return len(data)


class Decoder:
    """``decoder_interface<uint16_t>`` (decoder_interface.h:37-50)."""

    def __init__(self, config: CodecConfig, device: Union[str, torch.device] = "cuda"):
        _check(config)
        self.config = config
        self.device = torch.device(device)

    def decode(self, data: bytes, n_samples: int) -> np.ndarray:
        """Decodes exactly ``n_samples`` stored uint16 samples."""
        buf = np.frombuffer(bytes(data), np.uint8)
        padded = np.zeros(max(len(buf), 1) + 16, np.uint8)
        padded[: len(buf)] = buf
        d = torch.from_numpy(padded).to(self.device)
        out, status = decode_batch(self.config, d, [0], [len(buf)], [n_samples])
        _raise_status(int(status[0].item()))
        return out[:n_samples].cpu().numpy().view(np.uint16).copy()


def create_encoder(config: CodecConfig, device="cuda") -> Encoder:
    """``ricepp::create_encoder<uint16_t>`` (create_encoder.h:39-41)."""
    return Encoder(config, device)


def create_decoder(config: CodecConfig, device="cuda") -> Decoder:
    """``ricepp::create_decoder<uint16_t>`` (create_decoder.h:39-41)."""
    return Decoder(config, device)
